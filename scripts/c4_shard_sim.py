#!/usr/bin/env python3
"""Per-rank compute of the C4 view-sharded pipeline at world size N, on ONE
GPU, with the collectives replaced by replays of a world-1 run.

The world-1 run (all 32 views on this GPU) records every tensor its gathers
return.  Then, for each rank r of a world of N, the same ShardedPipeline runs
with a ReplayGather: each gather returns the recorded full tensor with rank
r's freshly computed block written into it, so every stage reads the same
(bit-exact) neighbour data it would read after a real all-gather, and the
rank does exactly its own share of the work.  Reports per rank the step time
(HIP events, same protocol as bench.py), the max over ranks, the world-1 time,
their ratio (the strong-scaling bound before communication), and the bytes
each gather delivers to a rank (what RCCL moves over xGMI per step).

    python scripts/c4_shard_sim.py [--world 8] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cl_multiview_stereo_amd import params, synth  # noqa: E402
from cl_multiview_stereo_amd.distributed import EngineBackend, ShardedPipeline, ViewGather  # noqa: E402,F401
from cl_multiview_stereo_amd.engine import CameraArray, Engine  # noqa: E402
from tests.replay_gather import RecordingGather, ReplayGather  # noqa: E402


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--save-rec", help="world-1 run only: save the recorded gathers here (torch.save) and exit")
    ap.add_argument("--load-rec", help="skip the world-1 run: replay the gathers saved by --save-rec")
    ap.add_argument("--bands", type=int, default=2, help="row bands of the proj all-gather (as at world > 1)")
    ap.add_argument("--only-rank", type=int, help="run this rank only (e.g. under rocprofv3 --kernel-trace)")
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
    be = EngineBackend(e, fused=True)
    if args.load_rec:
        saved = torch.load(args.load_rec, weights_only=True)
        rec = [t.cuda() for t in saved["rec"]]
        ref_filt, t1 = saved["filt"].cuda(), saved["t1"]
    else:
        rg = RecordingGather(V)
        sp1 = ShardedPipeline(be, st, cam, rg, pixel_cost="ncc", refine=True, filt=True, proj_bands=args.bands)
        ref_filt = sp1.run(rgbx).disp_filtered
        rec = list(rg.rec)
        t1 = timed(lambda: sp1.run(rgbx), args.steps, 1)
        if args.save_rec:
            torch.save({"rec": [t.cpu() for t in rec], "filt": ref_filt.cpu(), "t1": t1}, args.save_rec)
            print(json.dumps({"saved": args.save_rec, "world1_ms_per_step": round(t1, 3)}), flush=True)
            return
    n_gathers = len(rec)
    ranks = []
    for r in range(args.world) if args.only_rank is None else [args.only_rank]:
        g = ReplayGather(V, r, args.world, rec)
        sp = ShardedPipeline(be, st, cam, g, pixel_cost="ncc", refine=True, filt=True, proj_bands=args.bands)
        out = sp.run(rgbx)
        z0, z1 = g.block
        same = bool(torch.equal(out.disp_filtered.view(torch.int32), ref_filt[z0:z1].view(torch.int32)))
        g.bytes_in = 0
        g.events = []
        t = timed(lambda: sp.run(rgbx), args.steps, 0)
        cp = g.copy_ms() / args.steps
        g.events = None
        ranks.append({"rank": r, "views": [z0, z1], "ms_per_step": round(t, 3),
                      "replay_copy_ms_per_step": round(cp, 3), "compute_ms_per_step": round(t - cp, 3),
                      "filtered_bit_identical": same, "gather_bytes_in_per_step": g.bytes_in // args.steps})
    tmax = max(x["ms_per_step"] for x in ranks)
    cmax = max(x["compute_ms_per_step"] for x in ranks)
    print(json.dumps({"what": "C4 per-rank compute at world N, collectives replayed from a world-1 run (no comm)",
                      "world": args.world, "world1_ms_per_step": round(t1, 3), "max_rank_ms_per_step": tmax,
                      "compute_speedup_bound": round(t1 / tmax, 3),
                      "max_rank_compute_ms_per_step": cmax, "compute_speedup_bound_excl_replay": round(t1 / cmax, 3),
                      "note": "compute_ms = step - the replay's own device copies of the recorded gathers "
                              "(a real all-gather writes the caller's buffer in place)",
                      "gathers_per_step": n_gathers, "ranks": ranks}), flush=True)


if __name__ == "__main__":
    main()
