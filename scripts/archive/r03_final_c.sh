#!/usr/bin/env bash
# Round-3 measurement: kernel traces of the C2 SAD (reference-cost) step and of the C4 step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_sad -o run -- python3 bench.py \
  --cost sad --steps 5 --warmup 2 --no-cpu-baseline --no-sharded --no-reference-cost > gpurun_out/tr_sad.json 2> gpurun_out/tr_sad.err || exit 1
echo "sad done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr_c4 -o run -- python3 bench.py \
  --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-sharded --no-reference-cost > gpurun_out/tr_c4.json 2> gpurun_out/tr_c4.err || exit 1
echo done
