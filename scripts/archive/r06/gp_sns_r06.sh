# round-6: sweep.hip (superpixel sweeps, SAD band, WTA) with the SLP vectoriser off (sns) against the
# current build (base) -- parity under sns, then C4, C5 and ref
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06sn; mkdir -p $O
TAGS="base sns" TESTS="tests/test_gpu_parity.py tests/test_gpu_sad.py tests/test_gpu_ncc_configs.py" CONFIG=c4 ROUNDS=2 \
  ARGS="--no-reference-defaults --no-c3 --steps 10 --warmup 3" \
  timeout -k 10 900 bash scripts/ab_multi.sh > $O/ab_c4.txt 2>&1 || { cat $O/ab_c4.txt; exit 1; }
TAGS="base sns" CONFIG=c5 ROUNDS=2 ARGS="--no-reference-defaults --no-c3 --steps 10 --warmup 3" \
  timeout -k 10 600 bash scripts/ab_multi.sh > $O/ab_c5.txt 2>&1 || { cat $O/ab_c5.txt; exit 1; }
TAGS="base sns" CONFIG=ref ROUNDS=2 ARGS="--no-reference-defaults --no-c3 --steps 10 --warmup 3" \
  timeout -k 10 600 bash scripts/ab_multi.sh > $O/ab_ref.txt 2>&1 || { cat $O/ab_ref.txt; exit 1; }
cat $O/ab_c4.txt $O/ab_c5.txt $O/ab_ref.txt
