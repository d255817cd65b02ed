#!/usr/bin/env bash
# rocprofv3 kernel-trace + stats of one bench configuration (CONFIG, default
# c2), then separate PMC passes (FETCH_SIZE / WRITE_SIZE / SQ_INSTS_*) --
# counters never combined with other traces -- summarised into profiles/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
CONFIG=${CONFIG:-c2}
OUT=gpurun_out/prof_$CONFIG
mkdir -p $OUT
ARGS="--config $CONFIG ${BENCH_ARGS:---steps 5 --warmup 2 --no-cpu-baseline --no-sharded --no-reference-cost --no-reference-defaults --no-c3}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace_bench.json 2> $OUT/trace.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run -- python3 bench.py $ARGS > $OUT/pmc_fetch_bench.json 2> $OUT/pmc_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run -- python3 bench.py $ARGS > $OUT/pmc_write_bench.json 2> $OUT/pmc_write.err || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_MFMA -d $OUT/pmc_valu -o run -- python3 bench.py $ARGS > $OUT/pmc_valu_bench.json 2> $OUT/pmc_valu.err || exit $?
python3 scripts/summarize_prof.py $OUT ${TAG:-r02_$CONFIG} $CONFIG
