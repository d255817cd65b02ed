#!/usr/bin/env bash
# Kernel-time A/B of the default bench step: ab/libmvs_A.so (A) against the
# in-tree build (B), two interleaved rounds of a rocprofv3 --stats trace each;
# prints the average duration of the kernels matching KERNELS (regex).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab_k; rm -rf $O; mkdir -p $O
for r in 1 2; do
  for side in A B; do
    if [ $side = A ]; then export MVS_LIB=$PWD/ab/libmvs_A.so; else unset MVS_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$side$r -o run -- python3 bench.py \
      ${BENCH_ARGS:---steps 10 --warmup 2 --no-cpu-baseline --no-sharded --no-reference-cost} > $O/$side$r.json 2> $O/$side$r.err || exit 1
    f=$(find $O/$side$r -name "*kernel_stats.csv" | head -1)
    python3 - "$f" "$side$r" "${KERNELS:-assign|update}" <<'PY'
import csv, re, sys
for x in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], x["Name"]):
        n = re.sub(r"\(.*", "", x["Name"]).split("::")[-1]
        print(sys.argv[2], n, x["Calls"], round(float(x["AverageNs"]) / 1e3, 2), "us")
PY
  done
done
