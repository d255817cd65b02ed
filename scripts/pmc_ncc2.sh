#!/usr/bin/env bash
# HBM traffic + cache counters of the NCC sweep (scripts/bench_kernels.py ncc), one group per pass
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ncc2
rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES" "GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -d $OUT/p$i -o run -- python3 scripts/bench_kernels.py ${KERNELS:-ncc} > $OUT/p$i.txt 2>&1 || echo "pass $i ($grp) failed rc=$?"
done
python3 - <<'PY'
import sqlite3, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmc_ncc2/p*/**/*.db", recursive=True)):
    c = sqlite3.connect(f)
    for k, n, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
        k = k.replace("mvs::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if k.startswith("k_"):
            acc[(k, n)].append(v)
for (k, n), v in sorted(acc.items()):
    print(f"{k:36s} {n:24s} {sum(v)/len(v):18.1f}")
PY
