# round-6: C4's VERT matrix-core forms on the scalar-f32 build: the default choice (form 21 for the
# 5-NN lists: 32-level chunks, single-buffered) against forms 12 and 11 (16-level chunks)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ABARGS="--steps 10 --warmup 3" bash scripts/gpu_pass.sh r06vf abenv:c4:MVS_NCC_MFMA_V=12 abenv:c4:MVS_NCC_MFMA_V=11 || exit 1
cat gpurun_out/r06vf/abenv_c4.txt
