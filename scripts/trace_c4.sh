#!/usr/bin/env bash
# Kernel trace of the C4 view-sharded step on one GPU (all 32 views).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c4trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4trace -o run -- python3 bench.py \
  --config c4 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/c4trace/bench.json 2> gpurun_out/c4trace/err.txt || exit $?
f=$(find gpurun_out/c4trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -25
