#!/usr/bin/env python3
"""Summarise rocprofv3 output (rocpd SQLite) into profiles/<tag>_*.

    python scripts/summarize_prof.py <prof_dir> <tag> [<config>]

<prof_dir>/trace/*.db     --kernel-trace --stats   -> <tag>_kernel_stats.csv
<prof_dir>/pmc_fetch/*.db --pmc FETCH_SIZE          \
<prof_dir>/pmc_write/*.db --pmc WRITE_SIZE          -> <tag>_pmc.json, pmc_wta_<config>.json
<prof_dir>/pmc_valu/*.db  --pmc SQ_INSTS_VALU ...   -> pmc_ncc_<config>.json
(bench.py reads pmc_wta_<config>.json / pmc_ncc_<config>.json for the run's
own configuration only, shape-checked against <prof_dir>/trace_bench.json.)
FETCH_SIZE on gfx950 counts 128-B requests at 64 B for wide coalesced streaming
reads: it is doubled (MI355X_MICROARCH.md, HBM section).  WRITE_SIZE is exact
for 16-B-per-lane streaming stores.
"""
import csv
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def db(path):
    f = glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    return sqlite3.connect(f[0]) if f else None


def short(name):
    n = name.replace("mvs::ncc::(anonymous namespace)::", "").replace("mvs::(anonymous namespace)::", "")
    n = n.replace("void ", "")
    return n.split("(")[0].strip()


NCC_SOURCES = ("cl_multiview_stereo_amd/csrc/ncc.hip", "cl_multiview_stereo_amd/csrc/ncc_mfma.hip",
               "cl_multiview_stereo_amd/csrc/ncc_common.h")


def ncc_src_sha16(root=ROOT):
    """sha256 (16 hex digits) of the NCC sweep sources: bench.py compares it with
    the tree it runs from and marks a PMC-derived fraction stale on a mismatch."""
    import hashlib
    h = hashlib.sha256()
    for f in NCC_SOURCES:
        p = os.path.join(root, f)
        if os.path.exists(p):
            h.update(open(p, "rb").read())
    return h.hexdigest()[:16]


def fused_kernel(name):
    """The fused sweep + WTA kernels: k_ncc_volume<..., true, NB> and k_ncc_mfma<BW>."""
    return name.startswith("k_ncc_mfma") or (name.startswith("k_ncc_volume") and ", true" in name)


def main():
    src, tag = sys.argv[1], sys.argv[2]
    cfg = sys.argv[3] if len(sys.argv) > 3 else "c2"
    shape = {}
    try:
        b = json.load(open(os.path.join(src, "trace_bench.json")))
        shape = {"W": b["config"]["width"], "H": b["config"]["height"], "D": b["config"]["hypotheses"]}
    except (OSError, ValueError, KeyError):
        pass
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    c = db(os.path.join(src, "trace"))
    rows = list(c.execute("select name,total_calls,total_duration,average,percentage from top_kernels"))
    with open(os.path.join(out, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for r in rows:
            w.writerow([short(r[0]), r[1], round(r[2], 1), round(r[3], 1), round(r[4], 3)])
    pmc = defaultdict(dict)
    for counter, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write"), ("SQ_INSTS_VALU", "pmc_valu"),
                         ("SQ_INSTS_LDS", "pmc_valu"), ("SQ_INSTS_MFMA", "pmc_valu")):
        d = db(os.path.join(src, sub))
        if d is None:
            continue
        acc = defaultdict(list)
        scale, unit = (1024.0, "_bytes_per_launch") if counter.endswith("SIZE") else (1.0, "_per_launch")
        for name, val in d.execute("select kernel_name, value from counters_collection where counter_name=?",
                                   (counter,)):
            acc[short(name)].append(val * scale)  # FETCH/WRITE_SIZE are KB; SQ_INSTS_* wave-instructions
        for k, v in acc.items():
            pmc[k][counter + unit] = sum(v) / len(v)
            pmc[k]["launches"] = len(v)
    for k, v in pmc.items():
        if "WRITE_SIZE_bytes_per_launch" not in v and "FETCH_SIZE_bytes_per_launch" not in v:
            continue
        if "FETCH_SIZE_bytes_per_launch" in v:
            v["hbm_read_bytes_corrected"] = 2.0 * v["FETCH_SIZE_bytes_per_launch"]
        v["hbm_bytes_per_launch"] = v.get("hbm_read_bytes_corrected", 0.0) + v.get("WRITE_SIZE_bytes_per_launch", 0.0)
    json.dump(pmc, open(os.path.join(out, f"{tag}_pmc.json"), "w"), indent=1, sort_keys=True)
    wta = next((k for k in sorted(pmc) if k.startswith("k_wta")), None)
    if wta:
        json.dump({"kernel": wta, "source": f"profiles/{tag}_pmc.json",
                   "hbm_bytes_per_launch": pmc[wta]["hbm_bytes_per_launch"],
                   "note": "2 x FETCH_SIZE + WRITE_SIZE, separate --pmc passes", "config": cfg, **shape},
                  open(os.path.join(out, f"pmc_wta_{cfg}.json"), "w"), indent=1)
    ncc = [k for k in sorted(pmc) if k.startswith(("k_ncc_volume", "k_ncc_mfma")) and "SQ_INSTS_VALU_per_launch" in pmc[k]]
    if ncc:
        extra = {}
        # the fused sweep runs several reference views per launch
        # (mvs_ncc_wta_range_d): its VALU total over the pass divided by the
        # views that pass's bench process swept (bench.py profile_counts)
        try:
            counts = json.load(open(os.path.join(src, "pmc_valu_bench.json")))["profile_counts"]
            tot = sum(pmc[k]["SQ_INSTS_VALU_per_launch"] * pmc[k]["launches"] for k in ncc if fused_kernel(k))
            mf = sum(pmc[k].get("SQ_INSTS_MFMA_per_launch", 0.0) * pmc[k]["launches"] for k in ncc if fused_kernel(k))
            if counts.get("ncc_wta_views") and tot:
                extra = {"fused_valu_wave_insts_per_view": tot / counts["ncc_wta_views"],
                         "fused_views_in_pass": counts["ncc_wta_views"],
                         "fused_launches_in_pass": sum(pmc[k]["launches"] for k in ncc if fused_kernel(k))}
                if mf:
                    extra["fused_mfma_insts_per_view"] = mf / counts["ncc_wta_views"]
        except (OSError, ValueError, KeyError):
            pass
        json.dump({k: {"valu_wave_insts_per_launch": pmc[k]["SQ_INSTS_VALU_per_launch"],
                       "lds_wave_insts_per_launch": pmc[k].get("SQ_INSTS_LDS_per_launch"),
                       "launches": pmc[k]["launches"]} for k in ncc} | extra |
                  {"source": f"profiles/{tag}_pmc.json", "note": "SQ_INSTS_VALU / SQ_INSTS_LDS, own --pmc pass",
                   "config": cfg, "ncc_src_sha16": ncc_src_sha16(), **shape},
                  open(os.path.join(out, f"pmc_ncc_{cfg}.json"), "w"), indent=1)
    for r in rows[:8]:
        print(f"{short(r[0]):40s} calls={r[1]:5d} avg={r[3]:9.3f} us  {r[4]:6.2f}%")
    for k in sorted(pmc):
        if k.split("<")[0] in ("k_wta", "k_ncc_volume", "k_ncc_mfma", "k_cvt", "k_update_tiles", "k_assign", "k_box_stats"):
            print(k, {a: round(b / 1e6, 2) for a, b in pmc[k].items() if "bytes" in a})


if __name__ == "__main__":
    main()
