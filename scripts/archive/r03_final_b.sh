#!/usr/bin/env bash
# Round-3 measurement: one bench line per BASELINE configuration and the reference-cost line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${CONFIGS:-c3 c4 c5 ref}; do
  timeout -k 10 600 python3 bench.py --config $cfg --no-sharded --no-reference-cost > gpurun_out/r03c_bench_$cfg.json 2> gpurun_out/r03c_bench_$cfg.err || { tail -5 gpurun_out/r03c_bench_$cfg.err; exit 1; }
  echo "$cfg done"
done
timeout -k 10 600 python3 bench.py --cost sad --no-sharded --no-reference-cost > gpurun_out/r03c_bench_c2sad.json 2> gpurun_out/r03c_bench_c2sad.err || exit 1
echo done
