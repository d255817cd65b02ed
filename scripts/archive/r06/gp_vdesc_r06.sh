# round-6: the VERT matrix-core form's band DMA through buffer descriptors (vdesc)
# against the committed build (base), C4 with MVS_NCC_MFMA_V=1, and the scalar
# kernels (MVS_NCC_MFMA_V=0) -- parity under vdesc, then interleaved rounds
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06w; mkdir -p $O
TAGS="s=base/MVS_NCC_MFMA_V=0 v=base/MVS_NCC_MFMA_V=1 vd=vdesc/MVS_NCC_MFMA_V=1 vdesc" TESTS="tests/test_gpu_ncc_configs.py tests/test_gpu_c4.py" \
  CONFIG=c4 ROUNDS=2 ARGS="--no-reference-defaults --no-c3 --steps 10 --warmup 3" \
  timeout -k 10 1000 bash scripts/ab_multi.sh > $O/ab_c4.txt 2>&1 || { cat $O/ab_c4.txt; exit 1; }
cat $O/ab_c4.txt
