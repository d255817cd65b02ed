#!/usr/bin/env bash
# Kernel trace of the reference-defaults line (--config ref), for the
# 14.66 -> 17.2 ms question (Next 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03o; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --config ref \
  --steps 5 --warmup 2 --no-cpu-baseline --no-sharded > $O/tr.json 2> $O/tr.err || { tail -5 $O/tr.err; exit 1; }
f=$(find $O/tr -name "*kernel_stats.csv" | head -1); head -14 "$f"
