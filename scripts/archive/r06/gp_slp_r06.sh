# round-6: scalar f32 instead of packed v_pk_*_f32 outside the matrix-core sweep:
# asc (k_assign_tiles4, SLP off for slic.hip), ssc (k_sad_band's tap chain, SLP off
# for sweep.hip), noslp (the SLP vectoriser off for every file, sources as committed)
# against base (the committed build) -- the GPU suite under each, then C2, C3, ref, C1
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06u; mkdir -p $O
TAGS="base asc ssc noslp" TESTS="tests" CONFIG=c2 ROUNDS=3 ARGS="--no-reference-defaults --no-c3 --steps 20 --warmup 5" \
  timeout -k 10 1000 bash scripts/ab_multi.sh > $O/ab_c2.txt 2>&1 || { cat $O/ab_c2.txt; exit 1; }
TAGS="base noslp" CONFIG=c3 ROUNDS=2 ARGS="--no-reference-defaults --no-c3 --steps 20 --warmup 5" \
  timeout -k 10 600 bash scripts/ab_multi.sh > $O/ab_c3.txt 2>&1 || { cat $O/ab_c3.txt; exit 1; }
TAGS="base noslp" CONFIG=ref ROUNDS=2 ARGS="--no-reference-defaults --no-c3 --steps 10 --warmup 3" \
  timeout -k 10 600 bash scripts/ab_multi.sh > $O/ab_ref.txt 2>&1 || { cat $O/ab_ref.txt; exit 1; }
TAGS="base ssc noslp" CONFIG=c1 ROUNDS=2 ARGS="--no-reference-defaults --no-c3 --steps 50 --warmup 5" \
  timeout -k 10 600 bash scripts/ab_multi.sh > $O/ab_c1.txt 2>&1 || { cat $O/ab_c1.txt; exit 1; }
cat $O/ab_c2.txt $O/ab_c3.txt $O/ab_ref.txt $O/ab_c1.txt
