#!/usr/bin/env bash
# Round-3 closing pass (after the SAD loop split): the GPU suite and smoke, the driver's default bench
# line, the C4 line and its kernel trace, and the world-8 replay of C4.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03g_final; mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 600 python3 bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
echo default done
timeout -k 10 600 python3 bench.py --config c4 --no-sharded --no-reference-cost > $O/bench_c4.json 2> $O/bench_c4.err || { tail -5 $O/bench_c4.err; exit 1; }
echo c4 done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_c4 -o run -- python3 bench.py \
  --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-sharded --no-reference-cost > $O/tr_c4.json 2> $O/tr_c4.err || exit 1
echo c4 trace done
timeout -k 10 400 python3 scripts/c4_shard_sim.py --world 8 --steps 3 > $O/c4_shard_sim.json 2> $O/c4_shard_sim.err || exit 1
echo done
CONFIG=c2 TAG=r03g_c2 BENCH_ARGS="--steps 10 --warmup 3 --no-cpu-baseline --no-sharded --no-reference-cost" bash scripts/profile.sh > $O/profile_c2.log 2>&1 || { tail -5 $O/profile_c2.log; exit 1; }
mkdir -p $O/prof && cp profiles/archive/r03g_c2_* profiles/pmc_wta_c2.json profiles/pmc_ncc_c2.json $O/prof/
echo profile done
