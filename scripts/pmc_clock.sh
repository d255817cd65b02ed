#!/usr/bin/env bash
# Effective GPU clock per kernel: GRBM_GUI_ACTIVE cycles / dispatch duration
# (one --pmc pass over scripts/bench_kernels.py <kernels>)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_clock
rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $OUT -o run -- python3 scripts/bench_kernels.py ${KERNELS:-ncc wta fill} > $OUT/run.txt 2>&1 || exit $?
python3 - <<'PY'
import sqlite3, glob, collections
f = glob.glob("gpurun_out/pmc_clock/**/*.db", recursive=True)[0]
c = sqlite3.connect(f)
dur = {d: (e - s) for d, s, e in c.execute("select dispatch_id, start, end from rocpd_kernel_dispatch")}
acc = collections.defaultdict(list)
for d, k, n, v in c.execute("select dispatch_id, kernel_name, counter_name, value from counters_collection"):
    k = k.replace("mvs::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    acc[(k, n)].append((v, dur.get(d, 0)))
for (k, n), lst in sorted(acc.items()):
    v = sum(a for a, _ in lst) / len(lst); t = sum(b for _, b in lst) / len(lst)
    print(f"{k[:40]:40s} {n:16s} {v:14.0f} dur {t/1e3:9.1f} us  -> {v / max(t, 1):8.3f} cycles/ns")
PY
