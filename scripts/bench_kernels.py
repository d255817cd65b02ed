#!/usr/bin/env python3
"""Per-kernel timing at BASELINE config 2 (5-view 1080p, D=128, S=32, NCC 5x5).
Interleaved rounds in one process (cdna guide rule 24); prints a JSON dict."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from cl_multiview_stereo_amd import params, synth
from cl_multiview_stereo_amd.engine import CameraArray, Engine


def timeit(fn, reps=5):
    ts = []
    for _ in range(reps):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return min(ts), float(np.median(ts))


def main():
    which = sys.argv[1:] or ["all"]
    W, H, V, D = 1920, 1080, 5, 128
    e = Engine(0)
    stack, _ = synth.make_stack(W, H, 5, 1, 0, D - 1, 1.0, 0x5EED + 2)
    rgbx = torch.from_numpy(stack).cuda()
    levels = params.disparity_levels(0, D - 1, 1)
    vs, sn = params.flatten_subsets(params.neighbour_lists(5, 1, 4, 0))
    cam = CameraArray(5, 1.0, levels, vs, sn)
    lab, l8 = e.cvt(rgbx)
    box = e.box_stats(l8, 5)
    vol = e.ncc_volume(l8, box, cam, 2, 5)
    lv = e.levels_dev(cam)
    sp, lb = e.slic(lab, 32)
    rep = e.boundary(sp, lb, 32)
    torch.cuda.synchronize()
    out = {}
    run = lambda k: "all" in which or k in which
    if run("cvt"):
        out["cvt_5views"] = timeit(lambda: e.cvt(rgbx))
    if run("slic"):
        out["slic_5views_S32"] = timeit(lambda: e.slic(lab, 32))
    if run("boundary"):
        out["boundary"] = timeit(lambda: e.boundary(sp, lb, 32))
    if run("sweep_spixl"):
        out["sweep_spixl_5views"] = timeit(lambda: e.sweep_spixl(lab, sp, rep, cam, 32))
    if run("ncc"):
        out["ncc_volume_1view"] = timeit(lambda: e.ncc_volume(l8, box, cam, 2, 5, out=vol))
        out["ncc_volume_view0"] = timeit(lambda: e.ncc_volume(l8, box, cam, 0, 5, out=vol))
    if run("fused"):  # sweep + WTA in one kernel, no volume
        d1, c1 = e.ncc_wta(l8, box, cam, 2, 5)
        out["ncc_wta_fused_1view"] = timeit(lambda: e.ncc_wta(l8, box, cam, 2, 5, disp=d1, conf=c1))
        out["ncc_wta_fused_view0"] = timeit(lambda: e.ncc_wta(l8, box, cam, 0, 5, disp=d1, conf=c1))
        out["ncc_then_wta_1view"] = timeit(lambda: (e.ncc_volume(l8, box, cam, 2, 5, out=vol), e.wta(vol, lv)))
    if run("fill"):  # write floor: one pass of stores over a cost volume
        out["fill_volume"] = timeit(lambda: vol.fill_(1.0))
    if run("wta"):
        out["wta_1view"] = timeit(lambda: e.wta(vol, lv))
    if run("sad"):
        out["pixel_sad_1view"] = timeit(lambda: e.sweep_pixel_sad(lab, cam, 2, 3), reps=2)
    if run("refine"):
        out["refine_5views_S32"] = timeit(lambda: e.refine(sp, lb, rep, cam, 32), reps=2)
    print(json.dumps({k: [round(a, 4), round(b, 4)] for k, (a, b) in out.items()}), flush=True)


if __name__ == "__main__":
    main()
