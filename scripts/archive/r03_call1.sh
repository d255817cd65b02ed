#!/usr/bin/env bash
# round 3: default bench line + C2 trace/PMC refresh (k_wta<1,16>, fused sweep per view)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/r03_default.json 2> gpurun_out/r03_default.err || { echo "bench rc=$?"; tail -20 gpurun_out/r03_default.err; exit 1; }
cat gpurun_out/r03_default.json
CONFIG=c2 TAG=r03_c2 bash scripts/profile.sh || { echo "profile rc=$?"; exit 1; }
echo done
