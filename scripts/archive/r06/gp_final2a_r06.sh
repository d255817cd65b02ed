# round-6 final records, second session (part A: counters): PMC passes and kernel traces of the C2
# and C5 bench steps (the NCC sources changed: profiles/pmc_*.json carry their
# hash), the headline kernel's SQ counters, the GPU suite, smoke, the driver's
# bench command and every other configuration's line, a kernel trace of the
# driver's command with the trace-vs-line check, and the C4 replay bound.
# Summaries under gpurun_out/r06z; rocprof databases removed (64 MiB cap).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06z; mkdir -p $O
for C in c2 c5; do
  CONFIG=$C TAG=r06_$C timeout -k 10 900 bash scripts/profile.sh > $O/profile_$C.log 2>&1 || { tail -5 $O/profile_$C.log; exit 1; }
  tail -12 $O/profile_$C.log
  cp profiles/r06_${C}_pmc.json profiles/r06_${C}_kernel_stats.csv profiles/pmc_ncc_$C.json profiles/pmc_wta_$C.json $O/
  cp gpurun_out/prof_$C/trace_bench.json $O/trace_bench_$C.json
  python3 scripts/kstats.py gpurun_out/prof_$C/trace > $O/kernel_trace_$C.txt 2>&1
  rm -rf gpurun_out/prof_$C
done
KERNEL=k_ncc_mfma CONFIG=c2 TAG=mf5g BENCH_EXTRA="--no-reference-cost --no-reference-defaults --no-c3 --no-sharded" \
  timeout -k 10 600 bash scripts/pmc_kernel.sh > $O/pmc_mf5.txt 2>&1 || { tail -5 $O/pmc_mf5.txt; exit 1; }
rm -rf gpurun_out/pmc_kernel_mf5g
KERNEL=k_ncc_mfma CONFIG=c5 TAG=mf7g BENCH_EXTRA="--no-reference-cost --no-reference-defaults --no-c3 --no-sharded" \
  timeout -k 10 600 bash scripts/pmc_kernel.sh > $O/pmc_mf7.txt 2>&1 || { tail -5 $O/pmc_mf7.txt; exit 1; }
rm -rf gpurun_out/pmc_kernel_mf7g
du -sh gpurun_out
