#!/usr/bin/env bash
# NCC sweep A/B after peeling the first neighbour of each chunk (K = 5, EVEN):
# the GPU suite, then k_ncc_volume kernel time of the C2 step and the C2 /
# C5 / C4 lines, ab/libmvs_A.so (previous ncc.hip) vs the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03g_ncc; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
KERNELS=ncc_volume bash scripts/ab_kernels.sh > $O/ab_kernels_c2.txt 2>&1 || { tail -5 $O/ab_kernels_c2.txt; exit 1; }
cat $O/ab_kernels_c2.txt
CONFIG=c2 ARGS="--steps 20 --warmup 3 --no-reference-cost" bash scripts/ab_bench.sh > $O/ab_c2.txt 2>&1 || { tail -5 $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
CONFIG=c5 ARGS="--steps 3 --warmup 1" bash scripts/ab_bench.sh > $O/ab_c5.txt 2>&1 || { tail -5 $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
KERNELS=ncc_volume BENCH_ARGS="--config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-sharded --no-reference-cost" \
  bash scripts/ab_kernels.sh > $O/ab_kernels_c4.txt 2>&1 || { tail -5 $O/ab_kernels_c4.txt; exit 1; }
cat $O/ab_kernels_c4.txt
