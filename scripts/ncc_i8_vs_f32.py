"""What the i8 NCC definition costs in depth (CPU only).

The headline's cost is the build's own NCC on 8-bit intensities
(orc_l8: q = clamp(int(L * 2.55 + 0.5)), integer window sums; oracle/mvs_oracle.c
orc_ncc_volume).  This script runs the same sweep on the float L plane itself
(orc_ncc_volume_f32: no quantisation, double sums) over row bands of the C2
bench stack (5 views 1920 wide, levels 0..127, 4 horizontal neighbours, NCC
5x5; synth.make_stack seed 0x5EED + 2 = bench.py's) and reports, per band and
over all: the mean |d_i8 - d_f32| (px), the share of pixels whose disparity
differs and differs by more than 1 level, and -- for the centre view, whose
rendered ground truth is the canonical disparity map -- each definition's
mean error and > 1 px error rate against that ground truth.

    python scripts/ncc_i8_vs_f32.py [--rows 64] [--out profiles/r06/ncc_i8_vs_f32.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cl_multiview_stereo_amd import params, synth  # noqa: E402
from oracle import oracle as orc  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=64)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    W, H, aw, K, R = 1920, 1080, 5, 5, 2
    stack, gt = synth.make_stack(W, H, aw, 1, 0, 127, 1.0, 0x5EED + 2)
    levels = params.disparity_levels(0, 127, 1)
    vs, sn = params.flatten_subsets(params.neighbour_lists(aw, 1, 4, 0))
    bands = {"top": 0, "middle": H // 2 - a.rows // 2, "bottom": H - a.rows}
    res = {"what": "i8 NCC (the build's definition, the headline's cost) against the same NCC on float L "
                   "(orc_ncc_volume_f32), C2 bench stack, WTA disparities",
           "config": {"W": W, "views": aw, "levels": len(levels), "K": K, "neighbours": int(sn.max()),
                      "rows_per_band": a.rows, "seed": "0x5EED + 2 (bench.py c2)"}, "bands": {}}
    tot = {"n": 0, "l1": 0.0, "diff": 0, "diff_gt1": 0}
    gt_tot = {"n": 0, "i8_err": 0.0, "f32_err": 0.0, "i8_bad": 0, "f32_bad": 0}
    t0 = time.perf_counter()
    for name, y0 in bands.items():
        b0, b1 = max(0, y0 - R), min(H, y0 + a.rows + R)
        lab = orc.cvt(np.ascontiguousarray(stack[:, b0:b1]))
        q = orc.l8(lab)
        k0, k1 = y0 - b0, y0 - b0 + a.rows
        # rows whose 5x5 window lies inside the band (the full image's rows)
        k0i = k0 if y0 == 0 else max(k0, R)
        k1i = k1 if y0 + a.rows == H else min(k1, b1 - b0 - R)
        band = {"rows": f"{y0}..{y0 + a.rows - 1}", "views": {}}
        for z in range(aw):
            di, _ = orc.wta(orc.ncc_volume(q, levels, vs, sn, aw, 1.0, K, z), levels)
            df, _ = orc.wta(orc.ncc_volume_f32(lab, levels, vs, sn, aw, 1.0, K, z), levels)
            di, df = di[k0i:k1i], df[k0i:k1i]
            d = np.abs(di - df)
            v = {"l1_px": float(d.mean()), "differ_pct": float(100.0 * np.mean(d > 0)),
                 "differ_gt1_pct": float(100.0 * np.mean(d > 1))}
            tot["n"] += d.size
            tot["l1"] += float(d.sum())
            tot["diff"] += int(np.count_nonzero(d > 0))
            tot["diff_gt1"] += int(np.count_nonzero(d > 1))
            if z == aw // 2:  # the centre view: the rendered scene's own disparity map
                g = gt[b0:b1][k0i:k1i].astype(np.float32)
                ei, ef = np.abs(di - g), np.abs(df - g)
                v["vs_ground_truth"] = {"i8_mean_err_px": float(ei.mean()), "f32_mean_err_px": float(ef.mean()),
                                        "i8_bad_gt1_pct": float(100.0 * np.mean(ei > 1)),
                                        "f32_bad_gt1_pct": float(100.0 * np.mean(ef > 1))}
                gt_tot["n"] += ei.size
                gt_tot["i8_err"] += float(ei.sum())
                gt_tot["f32_err"] += float(ef.sum())
                gt_tot["i8_bad"] += int(np.count_nonzero(ei > 1))
                gt_tot["f32_bad"] += int(np.count_nonzero(ef > 1))
            band["views"][str(z)] = {k: (round(x, 4) if isinstance(x, float) else x) for k, x in v.items()}
        res["bands"][name] = band
        print(name, json.dumps(band["views"]), flush=True)
    n = tot["n"]
    res["all"] = {"pixels": n, "l1_px": round(tot["l1"] / n, 4), "differ_pct": round(100.0 * tot["diff"] / n, 3),
                  "differ_gt1_pct": round(100.0 * tot["diff_gt1"] / n, 3)}
    g = gt_tot["n"]
    res["centre_view_vs_ground_truth"] = {
        "pixels": g, "i8_mean_err_px": round(gt_tot["i8_err"] / g, 4), "f32_mean_err_px": round(gt_tot["f32_err"] / g, 4),
        "i8_bad_gt1_pct": round(100.0 * gt_tot["i8_bad"] / g, 3), "f32_bad_gt1_pct": round(100.0 * gt_tot["f32_bad"] / g, 3)}
    res["host_seconds"] = round(time.perf_counter() - t0, 1)
    print(json.dumps({k: res[k] for k in ("all", "centre_view_vs_ground_truth", "host_seconds")}))
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
