#!/usr/bin/env bash
# Kernel trace of one bench configuration: CONFIG (default ref), STEPS (3);
# prints the per-step kernel summary (scripts/trace_summary.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
C=${CONFIG:-ref}; N=${STEPS:-3}
O=gpurun_out/trace_$C; rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --config $C \
  --steps $N --warmup 0 --no-cpu-baseline --no-sharded > $O/bench.json 2> $O/err.txt || { tail -3 $O/err.txt; exit 1; }
python3 scripts/trace_summary.py $(find $O -name "*kernel_trace.csv" | head -1) $N
