#!/usr/bin/env python3
"""Per-kernel dispatch count / average / total from a rocprofv3 --kernel-trace
database (run_results.db): python3 scripts/kstats.py DB [name-substring ...]."""
import collections
import glob
import os
import sqlite3
import sys


def main():
    db = sys.argv[1]
    if os.path.isdir(db):  # a rocprofv3 -d directory: its (one) database
        db = sorted(glob.glob(os.path.join(db, "**", "*.db"), recursive=True))[-1]
    keys = sys.argv[2:]
    c = sqlite3.connect(db)
    acc = collections.OrderedDict()
    for n, s, e in c.execute("select name, start, end from kernels order by start"):
        n = n.replace("mvs::ncc::(anonymous namespace)::", "").replace("mvs::(anonymous namespace)::", "")
        n = n.replace("void ", "").split("(")[0][:70]
        if keys and not any(k in n for k in keys):
            continue
        acc.setdefault(n, []).append((e - s) / 1e3)
    for n, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
        print(f"{n:70s} {len(v):5d} {sum(v) / len(v):10.1f} us {sum(v) / 1e3:9.2f} ms")


if __name__ == "__main__":
    main()
