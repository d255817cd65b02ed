#!/usr/bin/env python3
"""What the superpixel sweep (k_sweep_spixl, clcode.cl:972-1069) must fetch.

For the bench workload (default C2: 5 views 1920x1080, S = 32, 128 levels,
4 horizontal neighbours) this replays the kernel's tap addressing on the
oracle's own SLIC output: per superpixel, its 25 reference taps
(cx + i stx, cy + j sty), and per level and neighbour the neighbour taps
(xr - d dx, yr).  It counts the distinct 64-B and 128-B sectors of the
float4 Lab rows each superpixel touches (summed over superpixels: the
traffic when nothing stays in L2 between superpixels) and over the whole
launch (the floor if L2 held every line), to set next to PMC FETCH_SIZE.

    python3 scripts/sweep_lines.py [c2|c5] > profiles/r05/sweep_lines_<cfg>.json
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cl_multiview_stereo_amd import params, synth  # noqa: E402
from oracle import oracle as orc  # noqa: E402

CFG = {"c2": (1920, 1080, 5, 32, 127), "c5": (4096, 3072, 5, 40, 255)}


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c2"
    W, H, aw, S, dmax = CFG[name]
    stack, _ = synth.make_stack(W, H, aw, 1, 0, dmax, 1.0, 0x5EED + 2)
    levels = params.disparity_levels(0, dmax, 1).astype(np.float32)
    vs, sn = params.flatten_subsets(params.neighbour_lists(aw, 1, 4, 0))
    outs = [orc.slic(stack[v], S) for v in range(aw)]
    sp = np.stack([o[1] for o in outs])
    lb = np.stack([o[2] for o in outs])
    rep = orc.boundary(sp, lb, S).astype(np.int32)
    per64 = per128 = 0
    glob64, glob128 = set(), set()
    taps = 0
    for z in range(aw):
        r = rep[z].reshape(-1, 8)
        bl = np.maximum(r[:, 0], np.maximum(r[:, 1], r[:, 2]))
        br = np.maximum(r[:, 5], np.maximum(r[:, 6], r[:, 7]))
        bt = np.maximum(r[:, 0], np.maximum(r[:, 3], r[:, 5]))
        bb = np.maximum(r[:, 2], np.maximum(r[:, 4], r[:, 7]))
        stx = np.maximum(1.0, 0.25 * (bl + br).astype(np.float32).astype(np.float64)).astype(np.float32)
        sty = np.maximum(1.0, 0.25 * (bt + bb).astype(np.float32).astype(np.float64)).astype(np.float32)
        c = sp[z].reshape(-1, 8)
        cx, cy = c[:, 1], c[:, 2]
        ii = np.repeat(np.arange(-2, 3), 5).astype(np.float32)  # tap order: i (x) outer, j (y) inner
        jj = np.tile(np.arange(-2, 3), 5).astype(np.float32)
        xr = (cx[:, None] + ii[None, :] * stx[:, None]).astype(np.int32)  # trunc toward 0 as (int)
        yr = (cy[:, None] + jj[None, :] * sty[:, None]).astype(np.int32)
        inr = (xr >= 0) & (yr >= 0) & (xr < W) & (yr < H)
        for n in range(int(sn[z])):
            v = int(vs[z, n])
            dx = float(v % aw - z % aw)
            fdx = (levels * np.float32(dx)).astype(np.float32)
            xp = (xr[:, :, None].astype(np.float32) - fdx[None, None, :]).astype(np.int32)  # [M, 25, D]
            yp = np.broadcast_to(yr[:, :, None], xp.shape)
            ok = inr[:, :, None] & (xp >= 0) & (xp < W)
            byte = (yp.astype(np.int64) * W + xp) * 16
            sec64 = np.where(ok, byte // 64, -1)
            sec128 = np.where(ok, byte // 128, -1)
            taps += int(ok.sum())
            for sec, which in ((sec64, 64), (sec128, 128)):
                flat = sec.reshape(sec.shape[0], -1)
                cnt = 0
                for row in flat:  # distinct sectors per superpixel
                    u = np.unique(row[row >= 0])
                    cnt += len(u)
                    (glob64 if which == 64 else glob128).update((v * 10**12 + u).tolist())
                if which == 64:
                    per64 += cnt * 64
                else:
                    per128 += cnt * 128
    out = {"config": name, "W": W, "H": H, "views": aw, "S": S, "levels": dmax + 1,
           "neighbour_taps_in_image": taps,
           "lab_bytes_all_views": aw * W * H * 16,
           "per_superpixel_distinct_64B_sectors_bytes": per64,
           "per_superpixel_distinct_128B_lines_bytes": per128,
           "whole_launch_distinct_64B_bytes": len(glob64) * 64,
           "whole_launch_distinct_128B_bytes": len(glob128) * 128,
           "note": "a superpixel's neighbour taps per (neighbour, tap row) span 127*|dx| + 4*stx columns of ONE row "
                   "of that view; rows differ between superpixels (cy + j*sty), so two superpixels share lines "
                   "only by chance"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
