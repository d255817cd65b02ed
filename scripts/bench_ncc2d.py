#!/usr/bin/env python3
"""NCC volume timing on a 2D camera array (C4's 8x4 grid, 5 nearest neighbours,
1080p, D=128): vertical shifts make the LDS bands taller than on a row array."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from cl_multiview_stereo_amd import params, synth  # noqa: E402
from cl_multiview_stereo_amd.engine import CameraArray, Engine  # noqa: E402
from bench_kernels import timeit  # noqa: E402

e = Engine(0)
aw, ah, W, H, D = 8, 4, 1920, 1080, 128
stack, _ = synth.make_stack(W, H, aw, ah, 0, D - 1, 1.0, 0x5EED + 4)
rgbx = torch.from_numpy(stack).cuda()
vs, sn = params.flatten_subsets(params.nearest_neighbours(aw, ah, 5))
cam = CameraArray(aw, 1.0, params.disparity_levels(0, D - 1, 1), vs, sn)
lab, l8 = e.cvt(rgbx)
box = e.box_stats(l8, 5)
vol = e.ncc_volume(l8, box, cam, 9, 5)
out = {f"ncc2d_view{z}": timeit(lambda: e.ncc_volume(l8, box, cam, z, 5, out=vol)) for z in (0, 9, 13)}
print(json.dumps({k: [round(a, 4), round(b, 4)] for k, (a, b) in out.items()}))
