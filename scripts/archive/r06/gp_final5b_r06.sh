# round-6 closing records after the ring sweep's one-wave default (part B): the GPU suite, smoke, the
# driver's line and every configuration's line, a kernel trace of the driver's command with the
# trace-vs-line check.  Summaries under gpurun_out/r06f5b; rocprof database removed (64 MiB cap)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06f5b; mkdir -p $O
bash scripts/gpu_pass.sh r06f5b tests smoke bench bench:c1 bench:c3 bench:c4 bench:c5 bench:ref || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/trace_drv -o run -- python3 bench.py --gpus 1 --steps 20 \
  --warmup 5 > $O/trace_driver_bench.json 2> $O/trace_drv.err || { tail -5 $O/trace_drv.err; exit 1; }
python3 scripts/kstats.py $O/trace_drv > $O/c2_driver_kernel_trace.txt 2>&1
python3 scripts/headline_kernel_check.py $O/trace_drv $O/trace_driver_bench.json 20 5 > $O/headline_check.json 2>&1
cat $O/headline_check.json
rm -rf $O/trace_drv
du -sh gpurun_out
