#!/usr/bin/env bash
# Closing pass with the concurrent headline: the GPU suite, smoke, the
# driver's default bench line (and a --serial line for comparison).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
echo default done
timeout -k 10 600 python3 bench.py --serial --no-cpu-baseline --no-sharded --no-reference-cost > $O/bench_serial.json 2> $O/bench_serial.err || { tail -5 $O/bench_serial.err; exit 1; }
echo serial done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py \
  --steps 10 --warmup 3 --no-cpu-baseline --no-sharded --no-reference-cost > $O/tr.json 2> $O/tr.err || exit 1
echo trace done
