# round-6 batch 2: the superpixel ring sweep with its chain interleaved (ring2)
# against HEAD (base): every GPU test under each build, interleaved C2 rounds;
# then C4's VERT matrix-core form vs the scalar kernels, and the C4 world-8 replay
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06e; mkdir -p $O
TAGS="base ring2" TESTS="tests" CONFIG=c2 ARGS="--no-reference-defaults --no-c3" \
  timeout -k 10 900 bash scripts/ab_multi.sh > $O/ab_c2.txt 2>&1 || { cat $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
bash scripts/gpu_pass.sh r06e abenv:c4:MVS_NCC_MFMA_V=12 || exit 1
timeout -k 10 600 python3 scripts/c4_shard_sim.py --world 8 --steps 3 > $O/c4_shard_sim.json 2> $O/c4_shard_sim.err || { tail -5 $O/c4_shard_sim.err; exit 1; }
tail -c 600 $O/c4_shard_sim.json
