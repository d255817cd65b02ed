#!/usr/bin/env bash
# GPU-box round trip: parity tests, then a short bench.  Every GPU step has its
# own time limit; a crash/abort/timeout stops the script (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export OMP_NUM_THREADS=${OMP_NUM_THREADS:-16}
timeout -k 10 ${TEST_TIMEOUT:-900} python -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ "${SKIP_BENCH:-0}" = "1" ]; then exit $rc; fi
timeout -k 10 ${BENCH_TIMEOUT:-420} python bench.py ${BENCH_ARGS:---steps 5 --warmup 2} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
echo "bench rc=$brc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
exit $brc
