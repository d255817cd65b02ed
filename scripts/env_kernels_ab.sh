#!/usr/bin/env bash
# Interleaved A/B of one environment setting on scripts/bench_kernels.py
# (A: VAR=V set, B: unset), 3 rounds:  KV=MVS_SWEEP_ORDER=view WHICH=sweep_spixl bash scripts/env_kernels_ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
VAR=${KV%%=*}
for r in 1 2 3; do
  A=$(env "$KV" timeout -k 10 120 python3 scripts/bench_kernels.py $WHICH 2>/dev/null) || { echo "A failed"; exit 1; }
  B=$(timeout -k 10 120 python3 scripts/bench_kernels.py $WHICH 2>/dev/null) || { echo "B failed"; exit 1; }
  echo "A($KV) $A"; echo "B(unset) $B"
done
