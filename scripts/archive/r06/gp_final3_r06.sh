# round-6 closing check after refine.hip's build flag: the GPU suite, smoke, the driver's line, C3 and C4
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_pass.sh r06f3 tests smoke bench bench:c3 bench:c4 || exit 1
