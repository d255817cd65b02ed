#!/usr/bin/env bash
# One GPU call, several steps, each under its own time limit; the first failing
# step ends the call (no GPU step runs after a fault, abort or time-out).
#   scripts/gpu_pass.sh TAG STEP [STEP ...]
# Steps:
#   tests            the -m gpu suite                       -> gpurun_out/TAG/gpu_tests.log
#   tests:EXPR       the -m gpu suite, -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            the driver's command (bench.py --gpus 1 --steps 20 --warmup 5) -> bench.json
#   bench:CFG        bench.py --config CFG --no-cpu-baseline  -> bench_CFG.json
#   ab:CFG           interleaved A/B (ab/libmvs_A.so vs the in-tree build), 2 rounds -> ab_CFG.txt
#   abenv:CFG:VAR=V  interleaved A/B of one environment setting (A: unset, B: VAR=V), 2 rounds
#   trace:CFG        rocprofv3 --kernel-trace --stats of bench.py --config CFG --steps 5
#   pmc:CFG          scripts/profile.sh's PMC passes for CFG (profiles/pmc_*_CFG.json)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
fail() { echo "FAILED: $1"; tail -25 "$2"; exit 1; }
for s in "$@"; do
  case $s in
    tests|tests:*)
      K=${s#tests}; K=${K#:}
      timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${K:+-k "$K"} \
        > $O/gpu_tests.log 2>&1 || fail "$s" $O/gpu_tests.log
      tail -1 $O/gpu_tests.log ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
        || fail bench $O/bench.err
      python3 scripts/bench_brief.py $O/bench.json ;;
    bench:*)
      C=${s#bench:}
      timeout -k 10 600 python3 bench.py --config $C --no-cpu-baseline --no-sharded > $O/bench_$C.json \
        2> $O/bench_$C.err || fail "$s" $O/bench_$C.err
      python3 scripts/bench_brief.py $O/bench_$C.json ;;
    ab:*)
      C=${s#ab:}
      for r in 1 2; do
        for side in A B; do
          if [ $side = A ]; then export MVS_LIB=$PWD/ab/libmvs_A.so; else unset MVS_LIB; fi
          timeout -k 10 300 python3 bench.py --config $C --no-cpu-baseline --no-sharded --no-reference-cost \
            --no-reference-defaults --no-c3 ${ABARGS:-} > $O/ab_$side.json 2> $O/ab_$side.err || fail "$s $side" $O/ab_$side.err
          python3 -c "import json;j=json.load(open('$O/ab_$side.json'));print('$C $side', j['ms_per_step'], j['value'])" \
            | tee -a $O/ab_$C.txt
        done
      done
      unset MVS_LIB ;;
    abenv:*)
      X=${s#abenv:}; C=${X%%:*}; KV=${X#*:}; VAR=${KV%%=*}
      for r in 1 2; do
        for side in A B; do
          if [ $side = A ]; then unset $VAR; else export "$KV"; fi
          timeout -k 10 300 python3 bench.py --config $C --no-cpu-baseline --no-sharded --no-reference-cost \
            --no-reference-defaults --no-c3 ${ABARGS:-} > $O/abenv_$side.json 2> $O/abenv_$side.err || fail "$s $side" $O/abenv_$side.err
          python3 -c "import json;j=json.load(open('$O/abenv_$side.json'));print('$C $KV $side', j['ms_per_step'], j['value'], (j.get('roofline_sweep') or {}).get('avg_ms_per_view'))" \
            | tee -a $O/abenv_$C.txt
        done
      done
      unset $VAR ;;
    trace:*)
      C=${s#trace:}
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_$C -o run -- python3 bench.py --config $C \
        --steps 5 --warmup 2 --no-cpu-baseline --no-sharded --no-reference-cost --no-reference-defaults --no-c3 \
        > $O/trace_$C.json 2> $O/trace_$C.err || fail "$s" $O/trace_$C.err
      python3 scripts/kstats.py $O/trace_$C > $O/trace_$C.txt 2>&1; head -12 $O/trace_$C.txt ;;
    pmc:*)
      C=${s#pmc:}
      CONFIG=$C timeout -k 10 900 bash scripts/profile.sh > $O/pmc_$C.log 2>&1 || fail "$s" $O/pmc_$C.log
      tail -5 $O/pmc_$C.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "gpu_pass $TAG done"
