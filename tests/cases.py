"""Seeded synthetic test cases shared by the CPU and GPU test suites."""
from __future__ import annotations

import numpy as np

from cl_multiview_stereo_amd import params, synth

# name, array (aw, ah), image (W, H), S, levels, bl, neighbourhood (nh, nv), seed
CASES = {
    "c3x1_s8": dict(aw=3, ah=1, W=100, H=70, S=8, dmin=0, dmax=15, bl=1.0, nh=1, nv=1, seed=11),
    "c3x3_s8": dict(aw=3, ah=3, W=96, H=72, S=8, dmin=2, dmax=17, bl=1.0359, nh=1, nv=1, seed=12),
    "c3x1_s16": dict(aw=3, ah=1, W=130, H=90, S=16, dmin=0, dmax=15, bl=1.0, nh=2, nv=0, seed=14),
    "c2x2_s12": dict(aw=2, ah=2, W=90, H=61, S=12, dmin=0, dmax=9, bl=1.0359, nh=1, nv=1, seed=19),
    "c5x1_s32": dict(aw=5, ah=1, W=200, H=150, S=32, dmin=0, dmax=31, bl=1.0, nh=4, nv=0, seed=17),
    "c2x1_s40": dict(aw=2, ah=1, W=250, H=170, S=40, dmin=0, dmax=7, bl=1.0, nh=1, nv=0, seed=18),
    # up to 14 neighbours per view: the refinement's > 8-view (one lane per triangle) path
    "c5x3_s16": dict(aw=5, ah=3, W=96, H=64, S=16, dmin=0, dmax=11, bl=1.0359, nh=2, nv=1, seed=20),
}

PIXEL_CASES = {
    "c2x1_pix": dict(aw=2, ah=1, W=64, H=48, dmin=0, dmax=31, bl=1.0, nh=1, nv=0, seed=15),
    "c2x2_pix": dict(aw=2, ah=2, W=48, H=40, dmin=0, dmax=9, bl=1.0359, nh=1, nv=1, seed=16),
    "c3x1_pix_odd": dict(aw=3, ah=1, W=37, H=29, dmin=0, dmax=12, bl=1.0, nh=2, nv=0, seed=21),
}


def build(c: dict):
    V = c["aw"] * c["ah"]
    stack, gt = synth.make_stack(c["W"], c["H"], c["aw"], c["ah"], c["dmin"], c["dmax"], c["bl"], c["seed"])
    levels = params.disparity_levels(c["dmin"], c["dmax"], c.get("inc", 1))
    vs, sn = params.flatten_subsets(params.neighbour_lists(c["aw"], c["ah"], c["nh"], c["nv"]))
    return dict(V=V, stack=stack, gt=gt, levels=levels, vs=vs, sn=sn)


def as_u32(t) -> np.ndarray:
    a = t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)
    return a.view(np.uint32)
