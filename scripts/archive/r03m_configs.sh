#!/usr/bin/env bash
# The other configurations with the concurrent default (c3, c5, ref, c1):
# each line's oracle check must stay bit-exact.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03m; mkdir -p $O
for c in c3 c5 ref c1; do
  timeout -k 10 400 python3 bench.py --config $c --steps 5 --warmup 2 > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  python3 -c "import json;j=json.load(open('$O/bench_$c.json'));d=j.get('depth_l1_vs_oracle') or {};print('$c', j['ms_per_step'], j['value'], j['config'].get('streams'), d.get('value'), d.get('bit_exact'))"
done
