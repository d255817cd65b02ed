#!/usr/bin/env bash
# Round-2 bench lines for every BASELINE configuration + the reference
# defaults, and a kernel trace of the default (driver) command.  Each GPU step
# has its own time limit; the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python bench.py "$@" > $O/b_$n.json 2> $O/b_$n.err || { echo "$n rc=$?"; tail -5 $O/b_$n.err; exit 1; }
  python -c "import json;j=json.load(open('$O/b_$n.json'));print('$n', j['ms_per_step'], j['value'], (j.get('depth_l1_vs_oracle') or {}).get('bit_exact'), (j.get('cpu_baseline') or {}).get('value'))"
}
run default 400
run c3 400 --config c3
run ref 400 --config ref
run c5 500 --config c5 --steps 5 --warmup 2
run c2sad 400 --config c2 --cost sad --steps 5 --warmup 2 --no-sharded
run c4 400 --config c4 --steps 3 --warmup 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py \
  --no-cpu-baseline > /dev/null 2> $O/trace.err || { echo "trace rc=$?"; exit 1; }
echo done
