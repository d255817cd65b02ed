#!/usr/bin/env bash
# rocprofv3 kernel-trace + stats of the default bench, then two separate PMC
# passes (FETCH_SIZE / WRITE_SIZE) -- counters never combined with other traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS=${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- python3 bench.py $ARGS > $OUT/pmc_fetch_bench.json 2> $OUT/pmc_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python3 bench.py $ARGS > $OUT/pmc_write_bench.json 2> $OUT/pmc_write.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS -d $OUT/pmc_valu -o run -- python3 bench.py $ARGS > $OUT/pmc_valu_bench.json 2> $OUT/pmc_valu.err || exit $?
find $OUT -name "*.csv" | head -20
