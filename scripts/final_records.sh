set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/r05_fin; mkdir -p $O
bash scripts/gpu_pass.sh r05_fin tests smoke bench || exit 1
CONFIG=c2 TAG=r05_c2 timeout -k 10 900 bash scripts/profile.sh > $O/pmc_c2.log 2>&1 || { tail -5 $O/pmc_c2.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace_drv -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/trace_driver_bench.json 2> $O/trace_drv.err || { tail -5 $O/trace_drv.err; exit 1; }
python3 scripts/kstats.py $O/trace_drv > $O/c2_driver_kernel_trace.txt 2>&1
echo final done
