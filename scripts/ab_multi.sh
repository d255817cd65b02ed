#!/usr/bin/env bash
# A/B/C... of ab/libmvs_<tag>.so builds in one GPU session:
#   TAGS="base x y" [ROUNDS=2] [CONFIG=c2] [TESTS="tests/test_gpu_ncc_configs.py"] scripts/ab_multi.sh
# first the parity tests under each build (stop at a failure), then interleaved
# bench rounds; prints ms/step and the fused sweep's ms per view.  A tag
# X=Y/NAME=VALUE runs build ab/libmvs_Y.so as tag X with NAME=VALUE in the env.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for spec in $TAGS; do
  t=${spec%%=*}; [ "$spec" != "$t" ] && continue
  if [ -n "${TESTS:-}" ]; then
    MVS_LIB=$PWD/ab/libmvs_$t.so timeout -k 10 600 python -m pytest $TESTS -q -x -m gpu -p no:cacheprovider \
      --timeout 300 --timeout-method thread > gpurun_out/ab_test_$t.log 2>&1
    rc=$?; echo "tests $t rc=$rc $(tail -1 gpurun_out/ab_test_$t.log)"
    [ $rc -eq 0 ] || exit $rc
  fi
done
for r in $(seq ${ROUNDS:-2}); do
  for spec in $TAGS; do
    t=${spec%%=*}; lib=$t; ex=""
    if [ "$spec" != "$t" ]; then rest=${spec#*=}; lib=${rest%%/*}; ex=${rest#*/}; fi
    env $ex MVS_LIB=$PWD/ab/libmvs_$lib.so timeout -k 10 300 python3 bench.py --config ${CONFIG:-c2} --no-cpu-baseline \
      --no-sharded --no-reference-cost ${ARGS:-} > gpurun_out/ab_$t.json 2> gpurun_out/ab_$t.err || { tail -3 gpurun_out/ab_$t.err; exit 1; }
    python3 -c "import json;j=json.load(open('gpurun_out/ab_$t.json'));rs=j.get('roofline_sweep',{});print('$t', 'ms/step', j['ms_per_step'], 'Mpix/s', j['value'], 'sweep ms/view', rs.get('avg_ms_per_view'), 'two-pass', j.get('two_pass_variant',{}).get('ms_per_step'))"
  done
done
