# round-6: the VERT matrix-core form on C4 (MVS_NCC_MFMA_V=1) re-measured on the current build, and the DBG probes
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06v; mkdir -p $O
ABARGS="--steps 10 --warmup 3" bash scripts/gpu_pass.sh r06v abenv:c4:MVS_NCC_MFMA_V=1 || exit 1
timeout -k 10 120 python3 scripts/ncc_mfma_probe.py > $O/probe_k5.txt 2>&1 || exit 1
timeout -k 10 300 python3 scripts/ncc_mfma_probe.py --k7 > $O/probe_k7.txt 2>&1 || exit 1
cat $O/abenv_c4.txt $O/probe_k5.txt $O/probe_k7.txt
