#!/usr/bin/env python3
"""Diagnostics for the cross-view filter at C4 (32 views): for sampled (reference,
pixel) pairs, how many largest-first candidates k_remove_incons_sel evaluates
and how many gathers its early exit leaves -- the data behind the filter's
cost.  Runs the C4 pipeline on one GPU up to the refined maps."""
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


def main():
    aw, ah, W, H = 8, 4, 1920, 1080
    e = Engine(0)
    st = params.Settings(spixl_size=32, array_width=aw, array_height=ah, min_disp=0, max_disp=127, inc=1, neib_hor=0,
                         neib_ver=0, bl_ratio=1.0, window=5, cost="ncc")
    stack, _ = synth.make_stack(W, H, aw, ah, 0, 127, 1.0, 0x5EED + 2)
    rgbx = torch.from_numpy(stack).cuda()
    pipe = Pipeline(e, st, W, H, view_subset=params.nearest_neighbours(aw, ah, 5), pixel_cost="ncc", refine=True)
    out = pipe.exe_pipeline(rgbx)
    full = out.disp_refined.contiguous()
    V = full.shape[0]
    proj, filt = e.filter(full, aw, 1.0, 1.0)
    torch.cuda.synchronize()
    fuse = 0.5
    g = torch.Generator(device="cpu").manual_seed(1)
    n = 4096
    ps = torch.randint(0, W * H, (n,), generator=g)
    rs = torch.randint(0, V, (n,), generator=g)
    pf = proj.reshape(V, -1)[:, ps.cuda()].T.cpu().numpy()  # [n][V] candidates
    fullc = full.reshape(V, -1)
    iters, gathers, stable_at = [], [], []
    for s in range(n):
        p, r = int(ps[s]), int(rs[s])
        x, y = p % W, p // W
        crx, cry = r % aw, r // aw
        pv = pf[s]
        cands = sorted(set(float(v) for v in pv if v != 0), reverse=True)
        it = g_used = 0
        found = None
        for d in cands:
            it += 1
            nz = pv[pv != 0]
            A = float(np.sum(np.where(np.abs(nz - np.float32(d)) > fuse, -1.0, 0.0) +
                             np.where(np.abs(nz - np.float32(d)) <= fuse, 1.0, 0.0)))
            stab = A
            j = 0
            cx = np.arange(V) % aw
            cy = np.arange(V) // aw
            xx = (x - np.round(np.float32(d) * (cx - crx).astype(np.float32))).astype(np.int64)
            yy = (y - np.round(np.float32(d) * (cy - cry).astype(np.float32))).astype(np.int64)
            inb = (xx >= 0) & (yy >= 0) & (xx < W) & (yy < H)
            idx = torch.from_numpy(np.where(inb, yy * W + xx, 0)).cuda()
            vals = fullc[torch.arange(V, device="cuda"), idx].cpu().numpy()
            for j in range(V):
                if not (stab + (V - j) >= 0):
                    break
                if inb[j]:
                    g_used += 1
                    diff = abs(float(vals[j]) - d)
                    stab += -1.0 if diff > fuse else (1.0 if diff < fuse else 0.0)
            if stab >= 0:
                found = it
                break
        iters.append(it)
        gathers.append(g_used)
        stable_at.append(found if found is not None else -1)
    iters, gathers = np.array(iters), np.array(gathers)
    res = {"samples": n, "iters_mean": float(iters.mean()), "iters_p50": float(np.median(iters)),
           "iters_p90": float(np.percentile(iters, 90)), "iters_max": int(iters.max()),
           "gathers_mean": float(gathers.mean()), "gathers_p90": float(np.percentile(gathers, 90)),
           "none_stable_frac": float(np.mean(np.array(stable_at) < 0)),
           "distinct_cands_mean": float(np.mean([len(set(v for v in row if v != 0)) for row in pf])),
           "first_stable_frac": float(np.mean(np.array(stable_at) == 1)),
           "wave_max_iters_mean_of_64": float(np.mean([iters[i:i + 64].max() for i in range(0, n, 64)]))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
