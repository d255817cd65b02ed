#!/usr/bin/env bash
# A/B timing of two builds of libmvs.so in one GPU session, interleaved:
#   scripts/ab.sh <kernels> [rounds]   A = ab/libmvs_A.so, B = the in-tree build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in $(seq ${2:-3}); do
  echo -n "A "; MVS_LIB=$PWD/ab/libmvs_A.so timeout -k 10 120 python scripts/bench_kernels.py $1 || exit 1
  echo -n "B "; timeout -k 10 120 python scripts/bench_kernels.py $1 || exit 1
done
