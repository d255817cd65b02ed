set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c
timeout -k 10 120 python3 scripts/ncc_mfma_probe.py > gpurun_out/r06c/probe_k5.txt 2>&1 || exit 1
timeout -k 10 300 python3 scripts/ncc_mfma_probe.py --k7 > gpurun_out/r06c/probe_k7.txt 2>&1 || exit 1
KERNEL=k_ncc_mfma CONFIG=c2 TAG=mf5 BENCH_EXTRA="--no-reference-cost --no-reference-defaults --no-c3 --no-sharded" timeout -k 10 600 bash scripts/pmc_kernel.sh > gpurun_out/r06c/pmc_mf5.txt 2>&1 || exit 1
KERNEL=k_ncc_mfma CONFIG=c5 TAG=mf7 BENCH_EXTRA="--no-sharded" timeout -k 10 900 bash scripts/pmc_kernel.sh > gpurun_out/r06c/pmc_mf7.txt 2>&1 || exit 1
cat gpurun_out/r06c/probe_k5.txt gpurun_out/r06c/probe_k7.txt
