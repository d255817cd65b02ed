#!/usr/bin/env bash
# Round-3 measurement: the driver's default bench line, then the C2 trace + PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python3 bench.py > gpurun_out/r03c_bench_default.json 2> gpurun_out/r03c_bench_default.err || { tail -5 gpurun_out/r03c_bench_default.err; exit 1; }
echo "default done"
CONFIG=c2 TAG=r03c_c2 bash scripts/profile.sh || exit 1
echo done
