# round-6: the VERT matrix-core form as C4's default -- the GPU suite, smoke, C4's line
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_pass.sh r06x tests smoke bench:c4 || exit 1
