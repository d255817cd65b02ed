#!/usr/bin/env bash
# rocprofv3 kernel trace of one bench configuration: scripts/trace_bench.sh <config> [steps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/tb_$1
rm -rf $OUT; mkdir -p $OUT
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --config $1 --steps ${2:-2} --warmup 1 --no-cpu-baseline > $OUT/bench.json 2> $OUT/err.log
