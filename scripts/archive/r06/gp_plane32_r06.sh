# round-6: the scalar NCC kernels' band DMA through buffer descriptors (default)
# vs 64-bit per-lane addresses (MVS_NCC_PLANE32=0) -- parity tests, then an
# interleaved A/B on C4 (tall vertical / diagonal bands, the scalar fused sweep)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06l; mkdir -p $O
bash scripts/gpu_pass.sh r06l "tests:scalar_band_dma or c4_geometry or every_ncc_variant or ncc_wta_range" || exit 1
ABARGS="--steps 10 --warmup 3" bash scripts/gpu_pass.sh r06l abenv:c4:MVS_NCC_PLANE32=0 || exit 1
cat $O/abenv_c4.txt
