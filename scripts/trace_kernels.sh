#!/usr/bin/env bash
# rocprofv3 kernel trace of scripts/bench_kernels.py <which...>; summarise
# locally with: python scripts/summarize_prof.py gpurun_out/kt <tag>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
rm -rf gpurun_out/kt
mkdir -p gpurun_out/kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/trace -o run -- python3 scripts/bench_kernels.py "$@" > gpurun_out/kt/out.json 2> gpurun_out/kt/err.log
