"""Failure pattern of the fused NCC sweep against the oracle on a C2-like
case (W 200, H 40, 5x1 array, 128 levels): which pixel classes differ."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from cl_multiview_stereo_amd import params, synth
from cl_multiview_stereo_amd.engine import CameraArray, Engine
from oracle import oracle as orc
e = Engine(0)
aw, W, H, dmax = 5, 200, 40, 127
stack, _ = synth.make_stack(W, H, aw, 1, 0, dmax, 1.0, 0x5EED + 9)
levels = params.disparity_levels(0, dmax, 1)
vs, sn = params.flatten_subsets(params.neighbour_lists(aw, 1, 4, 0))
cam = CameraArray(aw, 1.0, levels, vs, sn)
lab, l8 = e.cvt(torch.from_numpy(stack).cuda())
box = e.box_stats(l8, 5)
l8h = l8.cpu().numpy()
for z in (0, 2):
    fd, fc = e.ncc_wta(l8, box, cam, z, 5)
    print("variant", e.ncc_last_variant())
    vol = orc.ncc_volume(l8h, levels, vs, sn, aw, 1.0, 5, z)
    od, oc = orc.wta(vol, levels)
    g = fd.cpu().numpy()
    bad = np.argwhere(g != od)
    print(f"z{z}: {len(bad)} differ")
    if len(bad):
        ys, xs = bad[:, 0], bad[:, 1]
        print(" (x%4, y%4) classes:", sorted(set(zip((xs % 4).tolist(), (ys % 4).tolist()))))
        print(" rows:", sorted(set(ys.tolist()))[:20], "x%8:", sorted(set((xs % 8).tolist())))
        for (y, x) in bad[:6]:
            print(f"  ({x},{y}) gpu {g[y, x]} oracle {od[y, x]} costs oracle best {vol[:, y, x].min():.6f} at "
                  f"{vol[:, y, x].argmin()}; oracle cost at gpu level {vol[int(g[y, x]), y, x]:.6f}")
