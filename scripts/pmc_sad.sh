#!/usr/bin/env bash
# SQ / TCC counters of the per-pixel SAD sweep at C2 (MVS_SAD_KERNEL variant),
# one counter group per rocprofv3 pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export MVS_SAD_KERNEL=${MVS_SAD_KERNEL:-sys8x2}
OUT=gpurun_out/pmc_sad_$MVS_SAD_KERNEL
rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex k_sad_band -d $OUT/p$i -o run -- python3 bench.py \
    --config c2 --cost sad --steps 1 --warmup 0 --no-cpu-baseline --no-sharded > $OUT/p$i.txt 2>&1 || echo "pass $i failed rc=$?"
done
python3 - "$OUT" <<'PY'
import sqlite3, glob, collections, sys
acc = collections.defaultdict(list); durs = {}
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*.db", recursive=True)):
    c = sqlite3.connect(f)
    dur = {d: (e - s) for d, s, e in c.execute("select dispatch_id, start, end from rocpd_kernel_dispatch")}
    for d, k, n, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        k = k.replace("mvs::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        acc[(k, n)].append(v); durs.setdefault(k, []).append(dur.get(d, 0))
for (k, n), v in sorted(acc.items()):
    print(f"{k:32s} {n:26s} {sum(v)/len(v):18.1f}")
for k, v in durs.items():
    print(k, "avg dispatch us", sum(v) / len(v) / 1e3)
PY
