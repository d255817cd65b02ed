#!/usr/bin/env bash
# The driver's command shape (--steps 20 --warmup 5): concurrent headline
# (default) vs --serial, 4 interleaved rounds, headline pass only.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03l; mkdir -p $O
for r in 1 2 3 4; do
  for side in concurrent serial; do
    F=""; [ $side = serial ] && F="--serial"
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-sharded --no-reference-cost $F \
      > $O/$side$r.json 2> $O/$side$r.err || { tail -3 $O/$side$r.err; exit 1; }
    python3 -c "import json;j=json.load(open('$O/$side$r.json'));print('$side', j['ms_per_step'], j['value'], j.get('serial_variant',{}).get('ms_per_step'))"
  done
done
