#!/usr/bin/env python3
"""C4's cross-view filter split over the ranks of a world of N by image rows:
per rank, the time of its rows' projection + removal (all 32 reference
views), for contiguous row bands (today's split) and for cyclic splits (the
image cut into N * k equal bands, band b to rank b % N), each band one
proj + removal launch pair.  The maps are the world-1 refined disparity maps
of the C4 workload (scripts/c4_shard_sim.py's setup).

    python scripts/filter_band_balance.py [--world 8] [--reps 5]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cl_multiview_stereo_amd import params, synth  # noqa: E402
from cl_multiview_stereo_amd.distributed import EngineBackend, ShardedPipeline, ViewGather, all_blocks  # noqa: E402
from cl_multiview_stereo_amd.engine import CameraArray, Engine  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    aw, ah, W, H = 8, 4, 1920, 1080
    V = aw * ah
    e = Engine(0)
    st = params.Settings(spixl_size=32, array_width=aw, array_height=ah, min_disp=0, max_disp=127, inc=1, bl_ratio=1.0,
                         window=5, cost="ncc")
    stack, _ = synth.make_stack(W, H, aw, ah, 0, 127, 1.0, 0x5EED + 2)
    rgbx = torch.from_numpy(stack).cuda()
    mat, num = params.flatten_subsets(params.nearest_neighbours(aw, ah, 5))
    cam = CameraArray(aw, 1.0, params.disparity_levels(0, 127, 1), mat, num)
    sp = ShardedPipeline(EngineBackend(e, fused=True), st, cam, ViewGather(V), pixel_cost="ncc", refine=True,
                         filt=False)
    full = sp.run(rgbx).disp_refined.contiguous()
    fuse = st.fuse
    out = torch.zeros_like(full)
    s = torch.cuda.current_stream()

    def run_bands(bands):
        for ya, yb in bands:
            buf = torch.empty((V, yb - ya, W), dtype=torch.float32, device=full.device)
            e.proj_inv(full, aw, 1.0, 0, V, proj=buf, rows=(ya, yb), band=True)
            e.remove_inconsistency(full, buf, aw, 1.0, fuse, 0, V, out=out, rows=(ya, yb), band=True)

    def timed(bands):
        run_bands(bands)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(s)
        for _ in range(args.reps):
            run_bands(bands)
        ev[1].record(s)
        ev[1].synchronize()
        return ev[0].elapsed_time(ev[1]) / args.reps

    res = {"what": "C4 filter (proj + removal, 32 references) per rank of a row split", "world": args.world,
           "whole_image_ms": round(timed([(0, H)]), 3)}
    N = args.world
    for k in (1, 2, 4, 8):
        edges = all_blocks(H, N * k)
        per = [round(timed([edges[b] for b in range(r, N * k, N)]), 3) for r in range(N)]
        res[f"cyclic_k{k}" if k > 1 else "contiguous"] = {"per_rank_ms": per, "max_ms": max(per),
                                                          "mean_ms": round(sum(per) / N, 3)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
