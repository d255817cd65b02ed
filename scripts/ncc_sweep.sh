set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 -k "ncc or smoke" > gpurun_out/t.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/t.log
for d in 1 2 4; do MVS_NCC_DPW=$d timeout -k 10 120 python scripts/bench_kernels.py ncc wta || exit 1; done
