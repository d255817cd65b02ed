# round-6: refine.hip (removal walk, projection, propagation) with the SLP vectoriser off (rns: no
# v_pk_*_f32) against the current build (base) -- parity under rns, then C4 and C3
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06rn; mkdir -p $O
TAGS="base rns" TESTS="tests/test_gpu_c4.py tests/test_gpu_parity.py" CONFIG=c4 ROUNDS=2 \
  ARGS="--no-reference-defaults --no-c3 --steps 10 --warmup 3" \
  timeout -k 10 900 bash scripts/ab_multi.sh > $O/ab_c4.txt 2>&1 || { cat $O/ab_c4.txt; exit 1; }
TAGS="base rns" CONFIG=c3 ROUNDS=2 ARGS="--no-reference-defaults --no-c3 --steps 20 --warmup 5" \
  timeout -k 10 600 bash scripts/ab_multi.sh > $O/ab_c3.txt 2>&1 || { cat $O/ab_c3.txt; exit 1; }
cat $O/ab_c4.txt $O/ab_c3.txt
