#!/usr/bin/env python3
"""Cross-view filter at C4 (32 views, 8x4 array, 1080p): the refined
disparity maps of the C4 pipeline are computed once, then the filter
(k_proj_inv + the removal kernel) is timed for the whole array and for one
4-view shard, per variant (env knobs read per call), interleaved rounds.
Every variant's output is compared bit-for-bit with the first one's.
Prints one JSON dict of {variant: [min ms, median ms]}."""
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
    variants = sys.argv[1:] or ["MVS_FILTER_KERNEL=q", "MVS_FILTER_KERNEL=px"]
    aw, ah, W, H = 8, 4, 1920, 1080
    e = Engine(0)
    st = params.Settings(spixl_size=32, array_width=aw, array_height=ah, min_disp=0, max_disp=127, inc=1, neib_hor=0,
                         neib_ver=0, bl_ratio=1.0, window=5, cost="ncc")
    stack, _ = synth.make_stack(W, H, aw, ah, 0, 127, 1.0, 0x5EED + 2)
    rgbx = torch.from_numpy(stack).cuda()
    pipe = Pipeline(e, st, W, H, view_subset=params.nearest_neighbours(aw, ah, 5), pixel_cost="ncc", refine=True,
                    fused=True)
    full = pipe.exe_pipeline(rgbx).disp_refined.contiguous()
    torch.cuda.synchronize()
    res, ref = {}, {}
    for rnd in range(4):
        for v in variants:
            k, val = v.split("=")
            os.environ[k] = val
            for tag, (z0, z1) in (("all32", (0, 32)), ("shard4", (12, 16)), ("proj32", (0, 32))):
                s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                if tag == "proj32":
                    pj = e.proj_inv(full, aw, 1.0, z0, z1)
                    out = pj
                else:
                    pj, out = e.filter(full, aw, 1.0, 1.0, z0, z1)
                t.record()
                torch.cuda.synchronize()
                res.setdefault(f"{v}:{tag}", []).append(s.elapsed_time(t))
                o = np.concatenate([out[z0:z1].cpu().numpy().view(np.uint32).ravel(),
                                    pj[z0:z1].cpu().numpy().view(np.uint32).ravel()])
                if tag not in ref:
                    ref[tag] = o
                elif not np.array_equal(o, ref[tag]):
                    raise SystemExit(f"{v} {tag}: output differs from {variants[0]}")
            del os.environ[k]
    print(json.dumps({k: [round(min(v), 3), round(float(np.median(v)), 3)] for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
