#!/usr/bin/env python3
"""C4 NCC sweep diagnostics (8x4 array, 1080p, 128 levels, NCC 5x5): time of
the fused sweep + WTA of one reference view per neighbour direction (one
neighbour: horizontal, vertical, diagonal; and the 5-NN list) for the
automatic choice and for every forced (waves, levels per wave) variant.
Prints one JSON dict {case: {variant: [ms, chosen variant]}}."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cl_multiview_stereo_amd import params, synth  # noqa: E402
from cl_multiview_stereo_amd.engine import CameraArray, Engine  # noqa: E402


def main():
    aw, ah, W, H, K = 8, 4, 1920, 1080, 5
    e = Engine(0)
    stack, _ = synth.make_stack(W, H, aw, ah, 0, 127, 1.0, 0x5EED + 2)
    rgbx = torch.from_numpy(stack).cuda()
    lab, l8 = e.cvt(rgbx)
    box = e.box_stats(l8, K)
    levels = params.disparity_levels(0, 127, 1)
    V = aw * ah
    z = 9  # interior view (1, 1)
    cases = {
        "h1": {z: [z + 1]},
        "h2": {z: [z - 1, z + 1]},
        "v1": {z: [z + aw]},
        "v2": {z: [z - aw, z + aw]},
        "d1": {z: [z + aw + 1]},
        "knn5": {z: params.nearest_neighbours(aw, ah, 5)[z]},
        "corner0": {0: params.nearest_neighbours(aw, ah, 5)[0]},  # a neighbour two rows away
        "top1": {1: params.nearest_neighbours(aw, ah, 5)[1]},
        "edge8": {8: params.nearest_neighbours(aw, ah, 5)[8]},
    }
    if os.environ.get("CASES"):
        cases = {k: v for k, v in cases.items() if k in os.environ["CASES"].split(",")}
    variants = [(0, 0), (8, 4), (8, 2), (4, 4), (4, 2), (4, 1)]
    res = {}
    for name, nb in cases.items():
        z = next(iter(nb))  # the case's reference view
        lists = [nb.get(v, []) for v in range(V)]
        vs, sn = params.flatten_subsets(lists)
        cam = CameraArray(aw, 1.0, levels, vs, sn)
        ref = None
        for nw, dpw in variants:
            try:
                e.set_ncc_variant(nw, dpw)
                d, _ = e.ncc_wta(l8, box, cam, z, K)
            except Exception as ex:  # variant does not fit
                res.setdefault(name, {})[f"{nw}x{dpw}"] = str(ex)[:60]
                continue
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                d, _ = e.ncc_wta(l8, box, cam, z, K)
                t.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(t))
            dv = d.cpu().numpy()
            same = ref is None or np.array_equal(dv.view(np.uint32), ref.view(np.uint32))
            if ref is None:
                ref = dv
            res.setdefault(name, {})[f"{nw}x{dpw}"] = [round(min(ts), 4), e.ncc_last_variant(), bool(same)]
        e.set_ncc_variant()
        print(name, json.dumps(res[name]), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
