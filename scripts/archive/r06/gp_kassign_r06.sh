# round-6: the generic k_assign (S % 32 != 0: C5's S = 40, the reference defaults' S = 8) with
# k_assign_tiles4's fast candidate test (in-tree) against the committed build (ab/libmvs_A.so) --
# the GPU suite, then interleaved A/B on C5 and ref
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_pass.sh r06ka tests || exit 1
ABARGS="--steps 10 --warmup 3" bash scripts/gpu_pass.sh r06ka ab:c5 ab:ref ab:c5 || exit 1
cat gpurun_out/r06ka/ab_c5.txt gpurun_out/r06ka/ab_ref.txt
