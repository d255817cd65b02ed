#!/usr/bin/env python3
"""Cross-view filter at C4: how evenly the per-lane candidate walks of
k_remove_incons_q fill a wave, and how much sorting a block's pixels by their
candidate count before dealing them to waves would even them out.  For
sampled blocks of 256 consecutive pixels of one row and one reference view it
counts each pixel's gathers under the kernel's exit rule (in-image bounds) and
reports the wave cost (the max over its 64 lanes) for the natural order (4
waves of 64 consecutive pixels) against the nd-sorted order.  Prints JSON."""
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


def rnd(v):
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
    proj, _ = e.filter(full, aw, 1.0, 1.0)
    fullc = full.reshape(V, -1).cpu().numpy()
    projc = proj.reshape(V, -1).cpu().numpy()
    fuse = np.float32(0.5)
    rng = np.random.default_rng(3)
    nblk = int(os.environ.get("BLOCKS", "60"))
    cx, cy = np.arange(V) % aw, np.arange(V) // aw
    nat, srt, tot_g, pix = 0.0, 0.0, 0.0, 0
    lanes = []
    tiles = os.environ.get("TILES") == "1"
    tile_nat, tile_2d = 0.0, 0.0
    for _ in range(nblk):
        y = int(rng.integers(0, H - 8)) if tiles else int(rng.integers(0, H))
        xb = int(rng.integers(0, W // 256)) * 256
        r = int(rng.integers(0, V))
        work, nds = [], []
        # TILES=1: a 64 x 8 block of pixels (row-major), compared as 8 row waves
        # of 64 against 8 waves of 8 x 8 tiles
        pixels = [(xb + i % 64, y + i // 64) for i in range(512)] if tiles else [(x, y) for x in range(xb, xb + 256)]
        for x, y in pixels:
            p = y * W + x
            pv = projc[:, p]
            nz = pv[pv != 0]
            cands = sorted(set(float(v) for v in nz), reverse=True)
            nds.append(len(cands))
            g = 0
            for d in cands:
                d32 = np.float32(d)
                A = int(np.sum(np.abs(nz - d32) <= fuse)) * 2 - len(nz)
                xx = (x - rnd(d32 * (cx - cx[r]).astype(np.float32))).astype(np.int64)
                yy = (y - rnd(d32 * (cy - cy[r]).astype(np.float32))).astype(np.int64)
                inb = (xx >= 0) & (yy >= 0) & (xx < W) & (yy < H)
                left = int(inb.sum())
                if A + left < 0:
                    continue
                vals = fullc[np.arange(V), np.where(inb, yy * W + xx, 0)]
                dv = np.abs(vals - d32)
                vote = np.where(inb, np.where(dv > fuse, -1, np.where(dv < fuse, 1, 0)), 0)
                stab = A
                for j in range(V):
                    if stab + left < 0 or stab - left >= 0:
                        break
                    if inb[j]:
                        g += 1
                        left -= 1
                        stab += int(vote[j])
                if A + int(vote.sum()) >= 0:
                    break
            work.append(g)
        work = np.array(work, float)
        if tiles:
            blk = work.reshape(8, 64)
            tile_nat += blk.max(1).sum()
            tile_2d += blk.reshape(8, 8, 8).transpose(1, 0, 2).reshape(8, 64).max(1).sum()
            tot_g += work.sum()
            pix += 512
            continue
        lanes.append(work)
        nds = np.array(nds)
        tot_g += work.sum()
        pix += 256
        nat += sum(work[64 * w:64 * w + 64].max() for w in range(4))
        order = np.argsort(-nds, kind="stable")
        ws = work[order]
        srt += sum(ws[64 * w:64 * w + 64].max() for w in range(4))
        order2 = np.argsort(-work, kind="stable")  # oracle: sorted by the true work
        ws2 = work[order2]
    if tiles:
        print(json.dumps({"blocks": nblk, "lane_mean": tot_g / pix, "wave_cost_rows_64x1": tile_nat / (8 * nblk),
                          "wave_cost_tiles_8x8": tile_2d / (8 * nblk)}), flush=True)
        return
    # a capped first pass (each wave stops after K gathers per lane; lanes not
    # done are queued) plus a second pass over the queue, packed 64 to a wave:
    # wave cost per 64 pixels, in gathers, with `prep` gathers' worth of
    # restart cost per queued pixel
    allw = np.concatenate(lanes)
    waves = allw.reshape(-1, 64)
    split = {}
    for K in (8, 12, 16, 20, 24, 32):
        a_cost = np.minimum(waves.max(1), K).sum()
        ex = allw[allw > K] - K
        out = {}
        for prep in (0, 4, 8):
            q = rng.permutation(ex + prep)
            q = np.concatenate([q, np.zeros((-len(q)) % 64)]).reshape(-1, 64)
            out[f"prep{prep}"] = round(float((a_cost + q.max(1).sum()) / len(waves)), 2)
        out["queued_frac"] = round(float(len(ex) / len(allw)), 3)
        split[f"K{K}"] = out
    pct = {f"p{q}": float(np.percentile(allw, q)) for q in (50, 75, 90, 95, 99)}
    print(json.dumps({"blocks": nblk, "mean_gathers_per_pixel": tot_g / pix,
                      "wave_cost_natural": nat / (4 * nblk), "wave_cost_sorted_by_nd": srt / (4 * nblk),
                      "lane_mean": tot_g / pix, "lane_percentiles": pct, "capped_split": split}), flush=True)


if __name__ == "__main__":
    main()
