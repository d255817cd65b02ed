#!/usr/bin/env bash
# C2 step with the superpixel chain on a side stream (--concurrent) vs the
# default single stream, 3 interleaved rounds, after the NCC first-neighbour peel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03j; mkdir -p $O
for r in 1 2 3; do
  for side in serial concurrent; do
    F=""; [ $side = concurrent ] && F="--concurrent"
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-sharded --no-reference-cost $F \
      > $O/$side$r.json 2> $O/$side$r.err || { tail -3 $O/$side$r.err; exit 1; }
    python3 -c "import json;j=json.load(open('$O/$side$r.json'));print('$side', j['ms_per_step'], j['value'], j['depth_l1_vs_oracle']['bit_exact'] if j.get('depth_l1_vs_oracle') else None)"
  done
done
