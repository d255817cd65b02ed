#!/usr/bin/env bash
# SAD sweep A/B after the first-neighbour peel: parity tests of the
# per-pixel SAD kernels, then k_sad_band kernel time (rocprofv3, 2 interleaved
# rounds) and the C2 --cost sad step, ab/libmvs_A.so (previous) vs in-tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03i
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sad.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r03i/sad_tests.log 2>&1 || { tail -20 gpurun_out/r03i/sad_tests.log; exit 1; }
tail -2 gpurun_out/r03i/sad_tests.log
KERNELS=sad_band BENCH_ARGS="--config c2 --cost sad --steps 3 --warmup 1 --no-cpu-baseline --no-sharded --no-reference-cost" \
  bash scripts/ab_kernels.sh || exit 1
CONFIG=c2 ARGS="--cost sad --steps 5 --warmup 2 --no-reference-cost" bash scripts/ab_bench.sh || exit 1
