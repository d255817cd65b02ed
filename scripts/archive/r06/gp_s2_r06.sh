# (the parity tests of s2 and sal passed in the first run of this batch: gpurun_out/r06g/ab_c5.txt of that run)
# round-6 batch 4: s2 = HEAD's kernel + fewer scalar instructions per step
# (plane offsets in the plan records, the column -1 test skipped right of every
# shift, staging roles once per step), K = 7 double-buffered (NB = 3 opt-in);
# against sal (the same on the per-step-pitch kernel, K = 7 triple-buffered)
# and base (HEAD)
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r06g; mkdir -p $O
TAGS="s2 sal base s2nb3=s2/MVS_NCC_MFMA7_NB=3" CONFIG=c5 ROUNDS=2 \
  timeout -k 10 900 bash scripts/ab_multi.sh > $O/ab_c5.txt 2>&1 || { cat $O/ab_c5.txt; exit 1; }
cat $O/ab_c5.txt
TAGS="s2 sal base" CONFIG=c2 ARGS="--no-reference-defaults --no-c3" ROUNDS=3 \
  timeout -k 10 900 bash scripts/ab_multi.sh > $O/ab_c2.txt 2>&1 || { cat $O/ab_c2.txt; exit 1; }
cat $O/ab_c2.txt
