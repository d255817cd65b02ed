#!/usr/bin/env python3
"""Reproduce roofline_headline from a rocprofv3 kernel trace of the driver's
command (bench.py --gpus 1 --steps K --warmup W under --kernel-trace --stats):
the fused sweep's dispatches of the FIRST pass (warmup + timed steps of the
headline form, side stream included) are the first W + K launches of that
kernel in dispatch order; their average duration, the bench line's own
HIP-event average and the VALU fraction both give.

    python3 scripts/headline_kernel_check.py <trace_dir> <bench.json> [K W]
"""
import glob
import json
import os
import sqlite3
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    tdir, bj = sys.argv[1], sys.argv[2]
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    W = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    db = glob.glob(os.path.join(tdir, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    rows = list(c.execute("select k.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                          "join rocpd_info_kernel_symbol k on d.kernel_id = k.id order by d.start"))
    fused = [(s, e) for n, s, e in rows if "k_ncc_mfma" in n or ("k_ncc_volume" in n and ", true" in n)]
    head = fused[:W + K]
    timed = head[W:]
    avg_ms = sum(e - s for s, e in timed) / len(timed) / 1e6
    line = json.loads(open(bj).read().strip().splitlines()[-1])
    rh = line.get("roofline_headline") or {}
    views = line["config"]["views"]
    import bench
    pv = bench._valu_insts_fused_per_view(line["config"].get("name", "c2"), line["config"]["width"],
                                          line["config"]["height"], line["config"]["hypotheses"])
    issue = pv["insts"] - pv.get("mfma", 0.0)  # vector-ALU instructions only, as bench.py (SQ_INSTS_VALU counts MFMAs)
    frac = issue * views / (avg_ms * 1e-3) / bench.VALU_PEAK
    out = {"trace_dispatches_fused": len(fused), "headline_pass_launches": len(head),
           "trace_avg_ms_per_launch_timed": round(avg_ms, 4), "trace_avg_ms_per_view": round(avg_ms / views, 4),
           "trace_frac": round(frac, 4), "bench_avg_ms_per_view": rh.get("avg_ms_per_view"),
           "bench_frac": rh.get("frac"),
           "agreement": None if not rh.get("frac") else round(frac / rh["frac"], 4)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
