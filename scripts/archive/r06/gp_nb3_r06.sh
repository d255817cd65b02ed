# round-6 batch 3: the triple-buffered K = 7 matrix-core form (nb3 = the
# in-tree build), the per-step band pitch + K = 7 output mapping (pitch), and
# pitch + fewer scalar instructions per step (sal: plane offsets in the plan
# records, the column -1 test skipped right of every shift, staging roles
# decided once per step)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06f; mkdir -p $O
bash scripts/gpu_pass.sh r06f tests abenv:c5:MVS_NCC_MFMA7_NB=2 || exit 1
cat $O/abenv_c5.txt
TAGS="pitch sal nb3" TESTS="tests/test_gpu_ncc_configs.py tests/test_gpu_fullsize.py" CONFIG=c5 ROUNDS=2 \
  timeout -k 10 900 bash scripts/ab_multi.sh > $O/ab_c5_pitch.txt 2>&1 || { cat $O/ab_c5_pitch.txt; exit 1; }
cat $O/ab_c5_pitch.txt
TAGS="base pitch sal" CONFIG=c2 ARGS="--no-reference-defaults --no-c3" ROUNDS=2 \
  timeout -k 10 900 bash scripts/ab_multi.sh > $O/ab_c2_pitch.txt 2>&1 || { cat $O/ab_c2_pitch.txt; exit 1; }
cat $O/ab_c2_pitch.txt
