"""Time the fused NCC sweep of one C2 5-view launch (--k7: C5's 4096x3072,
256 levels, NCC 7x7) under MVS_NCC_MFMA_DBG (0 normal, 1 no compute, 2 no
band DMA) -- a timing probe, results ignored."""
import os, sys, time
import torch
sys.path.insert(0, ".")
from cl_multiview_stereo_amd import params, synth
from cl_multiview_stereo_amd.engine import CameraArray, Engine
e = Engine(0)
K7 = "--k7" in sys.argv
aw, W, H, D, K = (5, 4096, 3072, 256, 7) if K7 else (5, 1920, 1080, 128, 5)
stack, _ = synth.make_stack(W, H, aw, 1, 0, D - 1, 1.0, 0x5EED + 2)
levels = params.disparity_levels(0, D - 1, 1)
vs, sn = params.flatten_subsets(params.neighbour_lists(aw, 1, 4, 0))
cam = CameraArray(aw, 1.0, levels, vs, sn)
lab, l8 = e.cvt(torch.from_numpy(stack).cuda())
box = e.box_stats(l8, K)
for mode in ("0", "1", "2", "0"):
    os.environ["MVS_NCC_MFMA_DBG"] = mode
    for z0, z1 in (((0, 5), (2, 3)) if K7 else ((0, 5), (2, 3), (0, 1))):
        for _ in range(1 if K7 else 3):
            e.ncc_wta_range(l8, box, cam, z0, z1, K)
        torch.cuda.synchronize()
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        n = 3 if K7 else 10
        for _ in range(n):
            e.ncc_wta_range(l8, box, cam, z0, z1, K)
        t.record()
        torch.cuda.synchronize()
        print(f"K{K} dbg {mode} views {z0}..{z1 - 1}: {s.elapsed_time(t) / n / (z1 - z0):.4f} ms per view", flush=True)
