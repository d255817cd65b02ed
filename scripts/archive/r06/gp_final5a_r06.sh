# round-6 closing records after the ring sweep's one-wave default (part A): PMC passes and kernel traces of
# the C2 and C5 bench steps (profiles/pmc_*.json keep the NCC sources' hash).  Summaries under gpurun_out/r06f5
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06f5; mkdir -p $O
for C in c2 c5; do
  CONFIG=$C TAG=r06_$C timeout -k 10 900 bash scripts/profile.sh > $O/profile_$C.log 2>&1 || { tail -5 $O/profile_$C.log; exit 1; }
  cp profiles/r06_${C}_pmc.json profiles/r06_${C}_kernel_stats.csv profiles/pmc_ncc_$C.json profiles/pmc_wta_$C.json $O/
  python3 scripts/kstats.py gpurun_out/prof_$C/trace > $O/kernel_trace_$C.txt 2>&1
  rm -rf gpurun_out/prof_$C
done
du -sh gpurun_out
