# round-6 A/B batch: parity of each build, then interleaved C2 and C5 rounds
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06d
TAGS="base va vab" TESTS="tests/test_gpu_ncc_configs.py" CONFIG=c2 ARGS="--no-reference-defaults --no-c3" \
  timeout -k 10 900 bash scripts/ab_multi.sh > gpurun_out/r06d/ab_c2.txt 2>&1 || { cat gpurun_out/r06d/ab_c2.txt; exit 1; }
TAGS="base va" CONFIG=c5 ROUNDS=2 timeout -k 10 900 bash scripts/ab_multi.sh > gpurun_out/r06d/ab_c5.txt 2>&1 || { cat gpurun_out/r06d/ab_c5.txt; exit 1; }
cat gpurun_out/r06d/ab_c2.txt gpurun_out/r06d/ab_c5.txt
