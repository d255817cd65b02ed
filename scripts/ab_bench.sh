#!/usr/bin/env bash
# A/B of one bench configuration between ab/libmvs_A.so (A) and the in-tree
# build (B), interleaved: CONFIG (default c2), ARGS (extra bench.py flags).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2; do
  for side in A B; do
    if [ $side = A ]; then export MVS_LIB=$PWD/ab/libmvs_A.so; else unset MVS_LIB; fi
    timeout -k 10 300 python3 bench.py --config ${CONFIG:-c2} --no-cpu-baseline --no-sharded ${ARGS:-} \
      > gpurun_out/ab_$side.json 2> gpurun_out/ab_$side.err || { tail -3 gpurun_out/ab_$side.err; exit 1; }
    python3 -c "import json;j=json.load(open('gpurun_out/ab_$side.json'));print('$side', j['ms_per_step'], j['value'])"
  done
done
