#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAGS="cur sadlds" TESTS="tests/test_gpu_sad.py" CONFIG=c2 ARGS="--cost sad" ROUNDS=2 bash scripts/ab_multi.sh || exit 1
CONFIG=c2 TAG=r03b_c2 bash scripts/profile.sh || exit 1
echo done
