#!/usr/bin/env python3
"""Per-kernel calls / average / per-step total from a rocprofv3 --kernel-trace
CSV (run_kernel_trace.csv): python3 scripts/trace_summary.py CSV STEPS."""
import collections
import csv
import sys


def main():
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    acc = collections.defaultdict(list)
    iv = []
    for r in csv.DictReader(open(sys.argv[1])):
        n = r["Kernel_Name"].replace("mvs::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        acc[n].append((b - a) / 1e3)
        iv.append((a, b))
    tot = 0.0
    for n, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        tot += sum(v)
        print(f"{n:60s} {len(v):5d} {sum(v) / len(v):9.1f} us {sum(v) / steps / 1e3:7.3f} ms/step")
    print(f"{'total':60s} {'':5s} {'':12s} {tot / steps / 1e3:7.3f} ms/step")
    # device busy time (the union of the kernels' intervals) and the idle gaps
    # between them, over the whole trace
    iv.sort()
    busy, end, gaps = 0, None, []
    for a, b in iv:
        if end is None or a > end:
            if end is not None:
                gaps.append(a - end)
            busy += b - a
            end = b
        elif b > end:
            busy += b - end
            end = b
    span = iv[-1][1] - iv[0][0] if iv else 0
    print(f"{'busy (union of kernel intervals)':60s} {len(iv):5d} {'':12s} {busy / steps / 1e6:7.3f} ms/step")
    print(f"{'idle between kernels':60s} {len(gaps):5d} {'':12s} {sum(gaps) / steps / 1e6:7.3f} ms/step "
          f"(span {span / 1e6:.3f} ms)")


if __name__ == "__main__":
    main()
