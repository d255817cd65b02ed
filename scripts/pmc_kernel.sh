#!/usr/bin/env bash
# SQ counters of one kernel of a bench configuration, one counter group per pass:
#   KERNEL=k_propagate CONFIG=ref bash scripts/pmc_kernel.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_kernel${TAG:+_$TAG}
rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr" \
           "SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-include-regex "${KERNEL:-k_propagate}" -d $OUT/p$i -o run -- python3 bench.py --config ${CONFIG:-ref} --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_EXTRA:-} > $OUT/p$i.txt 2>&1 || echo "pass $i failed rc=$?"
done
OUT=$OUT python3 - <<'PY'
import sqlite3, glob, collections
acc = collections.defaultdict(list)
durs = {}
import os
for f in sorted(glob.glob(os.environ["OUT"] + "/p*/**/*.db", recursive=True)):
    c = sqlite3.connect(f)
    dur = {d: (e - s) for d, s, e in c.execute("select dispatch_id, start, end from rocpd_kernel_dispatch")}
    for d, k, n, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
        k = k.replace("mvs::ncc::(anonymous namespace)::", "").replace("mvs::(anonymous namespace)::", "")
        k = k.replace("void ", "").split("(")[0]
        acc[(k, n)].append(v)
        durs.setdefault(k, []).append(dur.get(d, 0))
for (k, n), v in sorted(acc.items()):
    print(f"{k:28s} {n:24s} {sum(v)/len(v):18.1f}")
for k, v in durs.items():
    print(k, "avg dispatch us", sum(v) / len(v) / 1e3)
PY
