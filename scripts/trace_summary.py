#!/usr/bin/env python3
"""Per-kernel calls / average / per-step total from a rocprofv3 --kernel-trace
CSV (run_kernel_trace.csv): python3 scripts/trace_summary.py CSV STEPS."""
import collections
import csv
import sys


def main():
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(sys.argv[1])):
        n = r["Kernel_Name"].replace("mvs::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        acc[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    tot = 0.0
    for n, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        tot += sum(v)
        print(f"{n:60s} {len(v):5d} {sum(v) / len(v):9.1f} us {sum(v) / steps / 1e3:7.3f} ms/step")
    print(f"{'total':60s} {'':5s} {'':12s} {tot / steps / 1e3:7.3f} ms/step")


if __name__ == "__main__":
    main()
