#!/usr/bin/env bash
# SAD sweep: parity tests, then the C2-shaped per-pixel SAD step per kernel
# variant (MVS_SAD_KERNEL), then a kernel trace of the default variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sad
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sad.py tests/test_gpu_ncc_configs.py -v --timeout 200 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/sad/tests.log 2>&1
rc=$?; tail -5 gpurun_out/sad/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for k in ${KINDS:-sys8x2 sys8 gather}; do
  MVS_SAD_KERNEL=$k timeout -k 10 200 python bench.py --config c2 --cost sad --steps 3 --warmup 1 --no-cpu-baseline \
    --no-sharded > gpurun_out/sad/b_$k.json 2> gpurun_out/sad/b_$k.err || exit $?
  python -c "import json;j=json.load(open('gpurun_out/sad/b_$k.json'));print('$k',j['ms_per_step'],j['value'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sad/trace -o run -- python3 bench.py --config c2 \
  --cost sad --steps 3 --warmup 1 --no-cpu-baseline --no-sharded > /dev/null 2> gpurun_out/sad/trace.err || exit $?
f=$(find gpurun_out/sad/trace -name "*kernel_stats.csv" | head -1); head -12 "$f"
