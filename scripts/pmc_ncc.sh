#!/usr/bin/env bash
# PMC counters of the kernels in scripts/bench_kernels.py (one counter group per pass)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ncc
mkdir -p $OUT
K=${KERNELS:-ncc}
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_EXP TA_BUSY_avr"; do
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp -d $OUT/p$i -o run -- python3 scripts/bench_kernels.py $K > $OUT/p$i.txt 2>&1 || echo "pass $i failed rc=$?"
done
python3 - <<'PY'
import sqlite3, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmc_ncc/p*/**/*.db", recursive=True)):
    c = sqlite3.connect(f)
    for k, n, v in c.execute("select kernel_name, counter_name, value from counters_collection"):
        k = k.replace("mvs::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        if k.startswith("k_"):
            acc[(k, n)].append(v)
for (k, n), v in sorted(acc.items()):
    print(f"{k:28s} {n:24s} {sum(v)/len(v):16.1f}")
PY
