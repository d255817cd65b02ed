# round-6: (1) the C2 step eager / eager with kernel timing / replayed from a HIP
# graph (scripts/probes/graph_step.py); (2) scalar f32 (no v_pk_*_f32, SLP
# vectoriser off for the file) in the scalar NCC kernels (nsc) and in
# k_assign_tiles4 (asc) against the committed build (base) -- parity, C2, C4
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06t; mkdir -p $O
timeout -k 10 300 python3 scripts/probes/graph_step.py --steps 20 --rounds 3 > $O/graph_step.txt 2>&1 || { tail -20 $O/graph_step.txt; exit 1; }
cat $O/graph_step.txt
TAGS="base nsc asc" TESTS="tests/test_gpu_ncc_configs.py tests/test_gpu_parity.py tests/test_gpu_c4.py" CONFIG=c2 ROUNDS=2 \
  ARGS="--no-reference-defaults --no-c3 --steps 20 --warmup 5" \
  timeout -k 10 900 bash scripts/ab_multi.sh > $O/ab_c2.txt 2>&1 || { cat $O/ab_c2.txt; exit 1; }
TAGS="base nsc asc" CONFIG=c4 ROUNDS=2 ARGS="--no-reference-defaults --no-c3 --steps 10 --warmup 3" \
  timeout -k 10 900 bash scripts/ab_multi.sh > $O/ab_c4.txt 2>&1 || { cat $O/ab_c4.txt; exit 1; }
cat $O/ab_c2.txt $O/ab_c4.txt
