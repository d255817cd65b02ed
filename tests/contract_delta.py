#!/usr/bin/env python3
"""How far is the pinned numerical definition (no FP contraction) from a build
that contracts as the reference's OpenCL build does by default?

The reference builds clcode.cl with no options, so mul+add pairs inside one
expression may fuse (OpenCL FP_CONTRACT ON; SURVEY 8c lists the fmuladd sites
in cvt, slic_distance_function, the sweep and propagate).  This script runs
the oracle restatement twice on the same synthetic stacks -- the pinned build
(gcc, -ffp-contract=off) and oracle/_build/liboracle_contract.so (clang,
-ffp-contract=on -mfma; the pinned exp/powr stay uncontracted) -- and reports
per configuration: Lab bits changed, SLIC label flips per view, superpixel
seed (s7) mismatches, and depth L1 between the two builds' disparity maps.
CPU only (checker infrastructure: it lives under tests/ because it loads the
oracle).  Writes profiles/contract_delta.json.

    python tests/contract_delta.py [--configs c1,c2,c3,ref]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import CONFIGS  # noqa: E402
from cl_multiview_stereo_amd import params, synth  # noqa: E402
from oracle import oracle as orc  # noqa: E402

PINNED = orc.LIB_PATH
CONTRACT = os.path.join(ROOT, "oracle", "_build", "liboracle_contract.so")


def use(path):
    orc._lib = C.CDLL(path)


def run_config(name, cfg):
    W, H, S, V = cfg["W"], cfg["H"], cfg["S"], cfg["aw"] * cfg["ah"]
    stack, _ = synth.make_stack(W, H, cfg["aw"], cfg["ah"], cfg["dmin"], cfg["dmax"], cfg["bl"], 0x5EED + 2)
    levels = params.disparity_levels(cfg["dmin"], cfg["dmax"], 1)
    vs, sn = params.flatten_subsets(params.neighbour_lists(cfg["aw"], cfg["ah"], cfg["nh"], cfg["nv"]))
    outs = {}
    for tag, path in (("pinned", PINNED), ("contract", CONTRACT)):
        use(path)
        t0 = time.perf_counter()
        o = [orc.slic(stack[v], S) if S > 1 else orc.grid(stack[v], 1) for v in range(V)]
        lab = np.stack([x[0] for x in o])
        sp = np.stack([x[1] for x in o])
        lb = np.stack([x[2] for x in o])
        rep = orc.boundary(sp, lb, S)
        sp = orc.sweep(lab, sp, rep, levels, vs, sn, cfg["aw"], cfg["bl"], S)
        r = dict(lab=lab, labels=lb, spixl=sp)
        if cfg["cost"] == "ncc":
            q = orc.l8(lab)
            r["disp"] = np.stack([orc.wta(orc.ncc_volume(q, levels, vs, sn, cfg["aw"], cfg["bl"], cfg["K"], z),
                                          levels)[0] for z in range(V)])
        elif cfg["cost"] == "sad":
            r["disp"] = orc.sweep_pixel_sad(lab, levels, vs, sn, cfg["aw"], cfg["bl"])
        if cfg.get("refine"):
            r["disp_refined"] = orc.refine(sp, lb, rep, vs, sn, cfg["aw"], cfg["bl"], S)["disp"]
            if cfg.get("filt"):
                r["disp_filtered"] = orc.filt(r["disp_refined"], cfg["aw"], cfg["bl"], 1.0)[1]
        r["seconds"] = time.perf_counter() - t0
        outs[tag] = r
    a, b = outs["pinned"], outs["contract"]
    res = {"workload": cfg["workload"], "views": V, "size": [W, H], "S": S,
           "lab_values_changed_frac": float(np.mean(a["lab"].view(np.uint32) != b["lab"].view(np.uint32))),
           "label_flips_per_view": [int(np.count_nonzero(a["labels"][v] != b["labels"][v])) for v in range(V)],
           "label_flip_frac": float(np.mean(a["labels"] != b["labels"])),
           "s7_mismatches": int(np.count_nonzero(a["spixl"][..., 7] != b["spixl"][..., 7])),
           "superpixels": int(a["spixl"][..., 7].size)}
    for k in ("disp", "disp_refined", "disp_filtered"):
        if k in a:
            res[k] = {"l1_px": float(np.abs(a[k] - b[k]).mean()),
                      "pixels_differing_frac": float(np.mean(a[k] != b[k])),
                      "max_abs_px": float(np.abs(a[k] - b[k]).max())}
    res["seconds"] = {"pinned": round(a["seconds"], 1), "contract": round(b["seconds"], 1)}
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2,c3,ref")
    args = ap.parse_args()
    if not os.path.exists(CONTRACT):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "all", "contract"], check=True)
    out = {"what": "pinned oracle (gcc -ffp-contract=off) vs the same restatement built with clang "
                   "-ffp-contract=on -mfma (the reference's OpenCL default); same synthetic stacks",
           "threads": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))}
    for name in args.configs.split(","):
        out[name] = run_config(name, CONFIGS[name])
        print(name, json.dumps(out[name]), flush=True)
    with open(os.path.join(ROOT, "profiles", "contract_delta.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
