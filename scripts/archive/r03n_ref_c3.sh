#!/usr/bin/env bash
# ref: round-start kernels (ab/libmvs_A.so) vs this build, 2 interleaved rounds
# (10 steps, 3 warmup); c3: concurrent headline vs --serial, 3 interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r03n; mkdir -p $O
CONFIG=ref ARGS="--steps 10 --warmup 3" bash scripts/ab_bench.sh > $O/ab_ref.txt 2>&1 || { tail -5 $O/ab_ref.txt; exit 1; }
cat $O/ab_ref.txt
for r in 1 2 3; do
  for side in concurrent serial; do
    F="--serial"; [ $side = concurrent ] && F="--concurrent"
    timeout -k 10 300 python3 bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline --no-sharded $F \
      > $O/c3_$side$r.json 2> $O/c3_$side$r.err || { tail -3 $O/c3_$side$r.err; exit 1; }
    python3 -c "import json;j=json.load(open('$O/c3_$side$r.json'));print('c3 $side', j['ms_per_step'], j['value'], j.get('serial_variant',{}).get('ms_per_step'))"
  done
done
