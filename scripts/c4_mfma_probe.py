#!/usr/bin/env python3
"""C4 geometry (8x4 array, 1080p, 128 levels, NCC 5x5): the fused sweep + WTA
of one reference view per neighbour direction (h1 / h2 / v1 / v2 / d1, the
5-NN list and a corner view's list) in the scalar kernels and in each
matrix-core VERT form (MVS_NCC_MFMA_V), plus the form-12 timing probes
(MVS_NCC_MFMA_DBG=1: no MFMA / finish, 2: no band DMA).  Prints one line per
case: {form: [ms, variant, bit-identical to the scalar result]}."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cl_multiview_stereo_amd import params, synth  # noqa: E402
from cl_multiview_stereo_amd.engine import CameraArray, Engine  # noqa: E402


def timed(e, l8, box, cam, z, K, reps=5):
    d, _ = e.ncc_wta(l8, box, cam, z, K)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        d, _ = e.ncc_wta(l8, box, cam, z, K)
        t.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(t))
    return min(ts), d.cpu().numpy()


def main():
    aw, ah, W, H, K = 8, 4, 1920, 1080, 5
    e = Engine(0)
    stack, _ = synth.make_stack(W, H, aw, ah, 0, 127, 1.0, 0x5EED + 2)
    lab, l8 = e.cvt(torch.from_numpy(stack).cuda())
    box = e.box_stats(l8, K)
    levels = params.disparity_levels(0, 127, 1)
    V = aw * ah
    z = 9  # interior view (1, 1)
    knn = params.nearest_neighbours(aw, ah, 5)
    cases = {"h1": {z: [z + 1]}, "h2": {z: [z - 1, z + 1]}, "v1": {z: [z + aw]}, "v2": {z: [z - aw, z + aw]},
             "d1": {z: [z + aw + 1]}, "knn5": {z: knn[z]}, "corner0": {0: knn[0]}}
    forms = [("scalar", {"MVS_NCC_MFMA_V": "0"}), ("22", {"MVS_NCC_MFMA_V": "22"}), ("21", {"MVS_NCC_MFMA_V": "21"}),
             ("12", {"MVS_NCC_MFMA_V": "12"}), ("11", {"MVS_NCC_MFMA_V": "11"}),
             ("12_nocompute", {"MVS_NCC_MFMA_V": "12", "MVS_NCC_MFMA_DBG": "1"}),
             ("12_nodma", {"MVS_NCC_MFMA_V": "12", "MVS_NCC_MFMA_DBG": "2"})]
    for name, nb in cases.items():
        zr = next(iter(nb))
        vs, sn = params.flatten_subsets([nb.get(v, []) for v in range(V)])
        cam = CameraArray(aw, 1.0, levels, vs, sn)
        res, ref = {}, None
        for fname, env in forms:
            for k in ("MVS_NCC_MFMA_V", "MVS_NCC_MFMA_DBG"):
                os.environ.pop(k, None)
            os.environ.update(env)
            try:
                ms, d = timed(e, l8, box, cam, zr, K)
            except Exception as ex:  # the form does not fit
                res[fname] = str(ex)[:60]
                continue
            v = e.ncc_last_variant()
            if ref is None:
                ref = d
            res[fname] = [round(ms, 4), [v[k] for k in ("DPW", "BW", "NB")],
                          bool(np.array_equal(d.view(np.uint32), ref.view(np.uint32)))]
        for k in ("MVS_NCC_MFMA_V", "MVS_NCC_MFMA_DBG"):
            os.environ.pop(k, None)
        print(name, json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
