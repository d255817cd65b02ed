#!/usr/bin/env bash
# A/B of the C4 filter passes (scripts/bench_filter.py) between ab/libmvs_A.so
# (A) and the in-tree build (B), interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for side in A B; do
    if [ $side = A ]; then export MVS_LIB=$PWD/ab/libmvs_A.so; else unset MVS_LIB; fi
    echo -n "$side "; timeout -k 10 300 python3 scripts/bench_filter.py ${VARIANTS:-MVS_FILTER_BOUND=1} 2>/dev/null || exit 1
  done
done
