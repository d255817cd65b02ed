#!/usr/bin/env bash
# SAD sweep A/B after the chunk/neighbour loop split: parity tests of the
# per-pixel SAD kernels, then k_sad_band kernel time (rocprofv3, 2 interleaved
# rounds) and the C2 --cost sad step, ab/libmvs_A.so (previous) vs in-tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03g
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_sad.py -x -q --timeout 200 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r03g/sad_tests.log 2>&1 || { tail -20 gpurun_out/r03g/sad_tests.log; exit 1; }
tail -2 gpurun_out/r03g/sad_tests.log
KERNELS=sad_band BENCH_ARGS="--config c2 --cost sad --steps 3 --warmup 1 --no-cpu-baseline --no-sharded --no-reference-cost" \
  bash scripts/ab_kernels.sh || exit 1
CONFIG=c2 ARGS="--cost sad --steps 5 --warmup 2 --no-reference-cost" bash scripts/ab_bench.sh || exit 1
# SAD kernel VALU count (SQ_INSTS_VALU) of the new build, and the stale C5 k_wta PMC record
CONFIG=c2 TAG=r03g_c2sad BENCH_ARGS="--cost sad --steps 3 --warmup 1 --no-cpu-baseline --no-sharded --no-reference-cost" \
  bash scripts/profile.sh || exit 1
mkdir -p gpurun_out/r03g/prof_sad && mv profiles/pmc_wta_c2.json gpurun_out/r03g/prof_sad/ 2>/dev/null; mv profiles/pmc_ncc_c2.json gpurun_out/r03g/prof_sad/ 2>/dev/null
cp profiles/archive/r03g_c2sad_* gpurun_out/r03g/prof_sad/ 2>/dev/null
CONFIG=c5 TAG=r03g_c5 BENCH_ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-sharded --no-reference-cost" bash scripts/profile.sh || exit 1
mkdir -p gpurun_out/r03g/prof_c5 && cp profiles/archive/r03g_c5_* profiles/pmc_wta_c5.json profiles/pmc_ncc_c5.json gpurun_out/r03g/prof_c5/ 2>/dev/null
echo all done
