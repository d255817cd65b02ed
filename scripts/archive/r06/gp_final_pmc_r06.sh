# round-6 final kernel: rocprofv3 kernel traces + PMC passes of the C2 and C5
# bench steps (scripts/profile.sh: traffic for `roofline`, VALU / MFMA counts
# for `roofline_headline`), the headline kernel's SQ counters (SALU, LDS bank
# conflicts, waits) and the MVS_NCC_MFMA_DBG compute / DMA probes.  The
# summaries are copied under gpurun_out/r06h and the rocprof databases removed
# (gpurun returns at most 64 MiB of gpurun_out/).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06h; mkdir -p $O
for C in c2 c5; do
  CONFIG=$C TAG=r06_$C timeout -k 10 900 bash scripts/profile.sh > $O/profile_$C.log 2>&1 || { tail -5 $O/profile_$C.log; exit 1; }
  tail -12 $O/profile_$C.log
  cp profiles/r06_${C}_pmc.json profiles/r06_${C}_kernel_stats.csv profiles/pmc_ncc_$C.json profiles/pmc_wta_$C.json $O/
  cp gpurun_out/prof_$C/trace_bench.json $O/trace_bench_$C.json
  python3 scripts/kstats.py gpurun_out/prof_$C/trace > $O/kernel_trace_$C.txt 2>&1
  rm -rf gpurun_out/prof_$C
done
KERNEL=k_ncc_mfma CONFIG=c2 TAG=mf5f BENCH_EXTRA="--no-reference-cost --no-reference-defaults --no-c3 --no-sharded" \
  timeout -k 10 600 bash scripts/pmc_kernel.sh > $O/pmc_mf5.txt 2>&1 || { tail -5 $O/pmc_mf5.txt; exit 1; }
rm -rf gpurun_out/pmc_kernel_mf5f
timeout -k 10 120 python3 scripts/ncc_mfma_probe.py > $O/probe_k5.txt 2>&1 || exit 1
timeout -k 10 300 python3 scripts/ncc_mfma_probe.py --k7 > $O/probe_k7.txt 2>&1 || exit 1
cat $O/probe_k5.txt $O/probe_k7.txt
du -sh gpurun_out
