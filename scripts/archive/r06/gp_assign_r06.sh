# round-6: k_assign_tiles4 trims (the lane's (x - cx)^2 once for its 4 pixels,
# the near-tie test as compares, v_min3 without canonicalisation; in-tree)
# against the committed build (ab/libmvs_A.so) -- parity tests, interleaved A/B on C2 (twice) and C3
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06r; mkdir -p $O
bash scripts/gpu_pass.sh r06r "tests:slic or assign or superpixel or pipeline or fullsize or c3" || exit 1
ABARGS="--steps 20 --warmup 5" bash scripts/gpu_pass.sh r06r ab:c2 ab:c2 ab:c3 || exit 1
cat $O/ab_c2.txt $O/ab_c3.txt
ABARGS="--steps 10 --warmup 3" bash scripts/gpu_pass.sh r06r abenv:c5:MVS_NCC_MFMA7_NB=3 || exit 1
cat $O/abenv_c5.txt
