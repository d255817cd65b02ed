# round-6: the superpixel chain on a side stream (MVS_BENCH_CONCURRENT=1) vs one stream, on the scalar-f32 build,
# interleaved, C2 (three calls of two rounds) and C3
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ABARGS="--steps 20 --warmup 5" bash scripts/gpu_pass.sh r06c abenv:c2:MVS_BENCH_CONCURRENT=1 abenv:c2:MVS_BENCH_CONCURRENT=1 \
  abenv:c2:MVS_BENCH_CONCURRENT=1 abenv:c3:MVS_BENCH_CONCURRENT=1 || exit 1
cat gpurun_out/r06c/abenv_c2.txt gpurun_out/r06c/abenv_c3.txt
