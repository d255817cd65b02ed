#!/usr/bin/env bash
# C4 view-sharded step: per-rank compute bound at world 8 (all ranks, replayed
# gathers, scripts/c4_shard_sim.py; SIM=0 skips it), then a kernel trace of ONE
# rank's step (RANK, default 7) replaying the gathers a world-1 run saved
# under /tmp.  The trace CSVs stay under gpurun_out/c4rank/trace
# (scripts/trace_summary.py reads the per-dispatch timeline from them).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/c4rank; rm -rf $O; mkdir -p $O
if [ "${SIM:-1}" != 0 ]; then
  timeout -k 10 300 python3 scripts/c4_shard_sim.py --world 8 --steps 3 > $O/sim.json 2> $O/sim.err || { tail -5 $O/sim.err; exit 1; }
  cat $O/sim.json
fi
timeout -k 10 300 python3 scripts/c4_shard_sim.py --save-rec /tmp/c4rec.pt > $O/save.json 2> $O/save.err || { tail -5 $O/save.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 scripts/c4_shard_sim.py \
  --load-rec /tmp/c4rec.pt --only-rank ${RANK:-7} --steps 5 > $O/rank.json 2> $O/rank.err || { tail -5 $O/rank.err; exit 1; }
cat $O/rank.json
f=$(find $O/trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-5 "$f" | head -30
t=$(find $O/trace -name "*kernel_trace.csv" | head -1); python3 scripts/trace_summary.py "$t" ${STEPS_IN_TRACE:-6} > $O/summary.txt; cat $O/summary.txt
rm -f /tmp/c4rec.pt
