#!/usr/bin/env bash
# GPU tests, then NCC/WTA kernel timing per variant (MVS_NCC_TH:MVS_NCC_DPW).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in ${VARIANTS:-16:4 8:4 8:2}; do
  echo "TH:DPW=$v"
  MVS_NCC_TH=${v%%:*} MVS_NCC_DPW=${v##*:} timeout -k 10 120 python scripts/bench_kernels.py ncc wta || exit 1
done
