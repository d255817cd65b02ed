# round-6: k_ncc_mfma's per-step bank shifts (odd pk rows; K = 7 also the odd-g
# stats rows), plan memoised -- parity tests, LDS conflict counters of both
# builds (ab/libmvs_A.so: the committed kernel), interleaved A/B on C5 and C2
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06n; mkdir -p $O
bash scripts/gpu_pass.sh r06n "tests:ncc or fullsize" || exit 1
for C in c2 c5; do
  for side in A B; do
    if [ $side = A ]; then export MVS_LIB=$PWD/ab/libmvs_A.so; else unset MVS_LIB; fi
    timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE \
      --kernel-include-regex k_ncc_mfma -d $O/pmc_${C}_$side -o run -- python3 bench.py --config $C --steps 1 --warmup 0 \
      --no-cpu-baseline --no-sharded --no-reference-cost --no-reference-defaults --no-c3 > $O/pmc_${C}_$side.txt 2>&1 \
      || { echo "pmc $C $side failed"; tail -5 $O/pmc_${C}_$side.txt; exit 1; }
    python3 - $O/pmc_${C}_$side $C $side <<'PY' | tee -a $O/pmc_lds.txt
import sqlite3, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*.db", recursive=True):
    c = sqlite3.connect(f)
    for k, n, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
        acc[(k.split("(")[0].split("::")[-1], n)].append(v)
for (k, n), v in sorted(acc.items()):
    print(sys.argv[2], sys.argv[3], k[:50], n, round(sum(v) / len(v), 1))
PY
    rm -rf $O/pmc_${C}_$side
  done
done
unset MVS_LIB
ABARGS="--steps 10 --warmup 3" bash scripts/gpu_pass.sh r06n ab:c5 || exit 1
ABARGS="--steps 20 --warmup 5" bash scripts/gpu_pass.sh r06n ab:c2 || exit 1
cat $O/pmc_lds.txt $O/ab_c5.txt $O/ab_c2.txt
