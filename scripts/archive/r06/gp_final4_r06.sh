# round-6 closing records: PMC passes on the final NCC sources (C2, C5), the GPU suite, smoke, the driver's
# line and every configuration's line.  Summaries under gpurun_out/r06f4
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06f4; mkdir -p $O
for C in c2 c5; do
  CONFIG=$C TAG=r06_$C timeout -k 10 900 bash scripts/profile.sh > $O/profile_$C.log 2>&1 || { tail -5 $O/profile_$C.log; exit 1; }
  cp profiles/r06_${C}_pmc.json profiles/r06_${C}_kernel_stats.csv profiles/pmc_ncc_$C.json profiles/pmc_wta_$C.json $O/
  python3 scripts/kstats.py gpurun_out/prof_$C/trace > $O/kernel_trace_$C.txt 2>&1
  rm -rf gpurun_out/prof_$C
done
bash scripts/gpu_pass.sh r06f4 tests smoke bench bench:c1 bench:c3 bench:c4 bench:c5 bench:ref || exit 1
du -sh gpurun_out
