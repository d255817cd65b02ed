#!/usr/bin/env bash
# One bench configuration with an environment knob off / on, interleaved:
# CONFIG, ENV=NAME, OFF=value, ON=value, ARGS (extra bench.py flags).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for v in "$OFF" "$ON"; do
    env "$ENV=$v" timeout -k 10 300 python3 bench.py --config ${CONFIG:-c2} --no-cpu-baseline --no-sharded ${ARGS:-} \
      > gpurun_out/abenv.json 2> gpurun_out/abenv.err || { tail -3 gpurun_out/abenv.err; exit 1; }
    python3 -c "import json;j=json.load(open('gpurun_out/abenv.json'));print('${CONFIG:-c2} $ENV=$v', j['ms_per_step'], j['value'])"
  done
done
