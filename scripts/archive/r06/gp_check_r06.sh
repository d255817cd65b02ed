# round-6: the GPU suite and the matrix-core DBG probes (compute / DMA split) on the current build
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06o; mkdir -p $O
bash scripts/gpu_pass.sh r06o tests smoke || exit 1
timeout -k 10 120 python3 scripts/ncc_mfma_probe.py > $O/probe_k5.txt 2>&1 || exit 1
timeout -k 10 300 python3 scripts/ncc_mfma_probe.py --k7 > $O/probe_k7.txt 2>&1 || exit 1
cat $O/probe_k5.txt $O/probe_k7.txt
