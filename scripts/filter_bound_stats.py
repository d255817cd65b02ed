#!/usr/bin/env python3
"""Cross-view filter at C4 (32 views): gathers per (reference, pixel) of the
largest-first candidate walk under three exit rules, on sampled pairs of the
C4 pipeline's refined maps (one GPU for the pipeline, numpy for the walk):

  v_all  -- the kernel's rule: give up once stab + (views not yet visited) < 0;
  v_in   -- the same bound over the IN-IMAGE views not yet visited (an
            out-of-image reprojection never votes), computed without gathers;
  v_both -- v_in plus a success exit once stab - (in-image views left) >= 0.

Every rule returns the same answer (the stability count is exact); only the
number of gathers differs.  Prints one JSON dict."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cl_multiview_stereo_amd import params, synth  # noqa: E402
from cl_multiview_stereo_amd.engine import Engine  # noqa: E402
from cl_multiview_stereo_amd.pipeline import Pipeline  # noqa: E402


def rnd(v):  # roundf as the kernels evaluate it (round_ha: exact for every float)
    v = v.astype(np.float32)
    return np.trunc(v + np.copysign(np.float32(0.49999997), v)).astype(np.float32)


def main():
    aw, ah, W, H = 8, 4, 1920, 1080
    e = Engine(0)
    st = params.Settings(spixl_size=32, array_width=aw, array_height=ah, min_disp=0, max_disp=127, inc=1, neib_hor=0,
                         neib_ver=0, bl_ratio=1.0, window=5, cost="ncc")
    stack, _ = synth.make_stack(W, H, aw, ah, 0, 127, 1.0, 0x5EED + 2)
    pipe = Pipeline(e, st, W, H, view_subset=params.nearest_neighbours(aw, ah, 5), pixel_cost="ncc", refine=True)
    out = pipe.exe_pipeline(torch.from_numpy(stack).cuda())
    full = out.disp_refined.contiguous()
    V = full.shape[0]
    proj, filt = e.filter(full, aw, 1.0, 1.0)
    fullc = full.reshape(V, -1).cpu().numpy()
    projc = proj.reshape(V, -1).cpu().numpy()
    fuse = np.float32(0.5)
    rng = np.random.default_rng(1)
    n = int(os.environ.get("SAMPLES", "3000"))
    ps = rng.integers(0, W * H, n)
    rs = rng.integers(0, V, n)
    cx, cy = np.arange(V) % aw, np.arange(V) // aw
    tot = {"v_all": 0, "v_in": 0, "v_both": 0}
    zero_gather_cands = cands_total = 0
    in_counts = []
    for s in range(n):
        p, r = int(ps[s]), int(rs[s])
        x, y = p % W, p // W
        pv = projc[:, p]
        nz = pv[pv != 0]
        cands = sorted(set(float(v) for v in nz), reverse=True)
        for d in cands:
            d32 = np.float32(d)
            diff = np.abs(nz - d32)
            A = int(np.sum(diff <= fuse)) * 2 - len(nz)
            xx = (x - rnd(d32 * (cx - cx[r]).astype(np.float32))).astype(np.int64)
            yy = (y - rnd(d32 * (cy - cy[r]).astype(np.float32))).astype(np.int64)
            inb = (xx >= 0) & (yy >= 0) & (xx < W) & (yy < H)
            vals = fullc[np.arange(V), np.where(inb, yy * W + xx, 0)]
            dv = np.abs(vals - d32)
            vote = np.where(inb, np.where(dv > fuse, -1, np.where(dv < fuse, 1, 0)), 0)
            n_in = int(inb.sum())
            in_counts.append(n_in)
            cands_total += 1
            res = {}
            for rule in tot:
                stab, g, left_in = A, 0, n_in
                for j in range(V):
                    left_all = V - j
                    if rule == "v_all":
                        if stab + left_all < 0:
                            break
                    else:
                        if stab + left_in < 0 or (rule == "v_both" and stab - left_in >= 0):
                            break
                    if inb[j]:
                        g += 1
                        left_in -= 1
                        stab += int(vote[j])
                tot[rule] += g
                res[rule] = stab >= 0 if rule == "v_all" else None
            if A + n_in < 0:
                zero_gather_cands += 1
            # the exact answer (all rules agree): stable iff A + sum(vote) >= 0
            if A + int(vote.sum()) >= 0:
                break
    print(json.dumps({"samples": n, "candidates": cands_total,
                      "gathers_per_pair": {k: v / n for k, v in tot.items()},
                      "candidates_rejected_without_gathers_frac": zero_gather_cands / max(1, cands_total),
                      "in_image_views_mean": float(np.mean(in_counts))}), flush=True)


if __name__ == "__main__":
    main()
