#!/usr/bin/env bash
# pmc_kernel.sh for two kernels of one configuration, outputs kept apart.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for k in ${KERNELS:-k_sweep_spixl k_proj_inv}; do
  KERNEL=$k bash scripts/pmc_kernel.sh > gpurun_out/pmc_$k.txt 2>&1 || exit 1
  cat gpurun_out/pmc_$k.txt
done
