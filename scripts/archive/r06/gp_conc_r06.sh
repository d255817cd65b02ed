# round-6: the superpixel chain on a side stream (MVS_BENCH_CONCURRENT=1) vs one
# stream, on the final kernels, interleaved, C2 and C3
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ABARGS="--steps 20 --warmup 5" bash scripts/gpu_pass.sh r06j abenv:c2:MVS_BENCH_CONCURRENT=1 || exit 1
cp gpurun_out/r06j/abenv_c2.txt gpurun_out/r06j/abenv_c2_conc.txt
bash scripts/gpu_pass.sh r06j abenv:c2:MVS_BENCH_CONCURRENT=1 || exit 1
ABARGS="--steps 20 --warmup 5" bash scripts/gpu_pass.sh r06j abenv:c3:MVS_BENCH_CONCURRENT=1 || exit 1
cat gpurun_out/r06j/abenv_c2.txt gpurun_out/r06j/abenv_c3.txt
