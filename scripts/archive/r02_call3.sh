#!/usr/bin/env bash
# Beer-Garden end-to-end run (mvs_cli vs the oracle) and the C2-shaped SAD line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/beer gpurun_out/sad
export TMPDIR=/tmp
timeout -k 10 400 python -u tests/beer_garden.py gpu > gpurun_out/beer/run.log 2>&1 || { echo "beer rc=$?"; tail -20 gpurun_out/beer/run.log; exit 1; }
tail -3 gpurun_out/beer/run.log
timeout -k 10 300 python bench.py --config c2 --cost sad --steps 5 --warmup 2 --no-sharded > gpurun_out/sad/b_c2_sad.json 2> gpurun_out/sad/b_c2_sad.err || { echo "sad bench rc=$?"; tail -20 gpurun_out/sad/b_c2_sad.err; exit 1; }
cat gpurun_out/sad/b_c2_sad.json
