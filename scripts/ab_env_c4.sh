#!/usr/bin/env bash
# C4 step (bench.py --config c4, no sharded line, no CPU baseline) with an
# environment knob off / on, interleaved: ENV=NAME OFF=value ON=value.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for v in "$OFF" "$ON"; do
    env "$ENV=$v" timeout -k 10 300 python3 bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-sharded \
      > gpurun_out/abc4.json 2> gpurun_out/abc4.err || { tail -3 gpurun_out/abc4.err; exit 1; }
    python3 -c "import json;j=json.load(open('gpurun_out/abc4.json'));print('$ENV=$v', j['ms_per_step'], j.get('two_pass_variant',{}).get('ms_per_step'))"
  done
done
