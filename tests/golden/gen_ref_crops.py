#!/usr/bin/env python3
"""Freeze small fixtures from the reference's OWN kept outputs (container only).

The reference keeps SLIC overlays drawn by clSLIC::draw_segmentation_lines
(clSLIC.cpp:447-478) over its real input images.  tests/ref_artifacts.py shows
that the oracle reproduces them:
  * results/slic output/green_new<k>.png (Images/Beer-Garden/img<k>.png) with
    the active candidate loop (search 0, clcode.cl:474-494), and
  * results/blue_i<k>.png (Images/c<k>f1.png) with the 3x3 loop behind the
    comment switch (search 1, clcode.cl:496-516),
both at main()'s settings (S 8, weight 0.6, 5 iterations, clMVDE.cpp:14-36).

SLIC is local: a crop whose origin lies on the S grid yields, more than 40 px
inside its edges, exactly the labels of the full-image run (checked here for
every crop).  So each fixture holds a 160 x 160 crop of the input and the
reference overlay's boundary mask over the crop's 80 x 80 interior -- data
taken from the reference's files, no reference source.  The tests run the
oracle (CPU) and the HIP kernels (GPU) on the crop and require the interior
masks to equal the reference's bit for bit.

    python tests/golden/gen_ref_crops.py   ->  tests/golden/ref_overlay_crops.npz
    python tests/golden/gen_ref_crops.py --residual  ->  tests/golden/ref_overlay_residual.npz
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as orc  # noqa: E402
from tests.ref_artifacts import INNER, boundary_mask, load_rgb, overlay_mask, rgbx_of  # noqa: E402

SZ, MG, S = 160, 40, 8
CROPS = [  # family, search, input, overlay, (y0, x0) on the S grid
    ("green_new", 0, "Images/Beer-Garden/img0.png", "results/slic output/green_new0.png", (400, 800)),
    ("green_new", 0, "Images/Beer-Garden/img4.png", "results/slic output/green_new4.png", (640, 1200)),
    ("green_new", 0, "Images/Beer-Garden/img8.png", "results/slic output/green_new8.png", (160, 320)),
    ("blue_i", 1, "Images/c0f1.png", "results/blue_i0.png", (480, 880)),
    ("blue_i", 1, "Images/c7f1.png", "results/blue_i7.png", (240, 1440)),
    ("blue_i", 1, "Images/c14f1.png", "results/blue_i14.png", (560, 1040)),
]


def main():
    out = {}
    inner = np.s_[MG:SZ - MG, MG:SZ - MG]
    for i, (fam, search, inp, ov, (y0, x0)) in enumerate(CROPS):
        assert y0 % S == 0 and x0 % S == 0
        rgb = load_rgb(inp)
        ref = overlay_mask(load_rgb(ov), rgb)
        _, _, lb_full = orc.slic(rgbx_of(rgb), S, search=search)
        full = boundary_mask(lb_full)
        crop = np.ascontiguousarray(rgb[y0:y0 + SZ, x0:x0 + SZ])
        _, _, lb = orc.slic(rgbx_of(crop), S, search=search)
        got = boundary_mask(lb)[inner]
        want = ref[y0:y0 + SZ, x0:x0 + SZ][inner]
        assert (got == full[y0:y0 + SZ, x0:x0 + SZ][inner]).all(), (inp, "crop interior != full-image run")
        assert (got == want).all(), (inp, "oracle != reference overlay on this crop")
        print(f"{fam} {inp} @({y0},{x0}): interior boundary fraction {want.mean():.3f}, oracle == reference")
        out[f"rgb{i}"] = crop
        out[f"mask{i}"] = want
        out[f"meta{i}"] = np.array([search, y0, x0, MG], np.int32)
        out[f"src{i}"] = np.array(f"{fam}|{inp}|{ov}")
    assert INNER is not None
    np.savez_compressed(os.path.join(HERE, "ref_overlay_crops.npz"), n=np.int32(len(CROPS)), **out)
    print("wrote", os.path.join(HERE, "ref_overlay_crops.npz"))


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


# ---- residual crops (round 4): where the oracle does NOT reproduce the overlay
# The crops above were chosen where the oracle equals the reference; the
# residual (115 boundary pixels of 18.6 M on green_new) is then never
# seen by the fixture tests.  These crops are centred on the densest residual
# clusters of green_new0 / green_new4 and keep the mismatch count the oracle
# leaves there, so the tests assert the residual instead of selecting it away.
def residual_crops(views=(0, 4), per_view=1):
    out = {}
    inner = np.s_[MG:SZ - MG, MG:SZ - MG]
    i = 0
    for k in views:
        inp, ov = f"Images/Beer-Garden/img{k}.png", f"results/slic output/green_new{k}.png"
        rgb = load_rgb(inp)
        ref = overlay_mask(load_rgb(ov), rgb)
        _, _, lb_full = orc.slic(rgbx_of(rgb), S, search=0)
        full = boundary_mask(lb_full)
        mism = np.zeros(full.shape, bool)
        mism[INNER] = full[INNER] != ref[INNER]
        H, W = mism.shape
        # 80 x 80 interior windows on the S grid, the one holding most mismatches
        cs = np.pad(mism.cumsum(0).cumsum(1), ((1, 0), (1, 0)))
        best = []
        for y0 in range(0, H - SZ + 1, S):
            for x0 in range(0, W - SZ + 1, S):
                a, b = y0 + MG, x0 + MG
                n = cs[a + 80, b + 80] - cs[a, b + 80] - cs[a + 80, b] + cs[a, b]
                best.append((int(n), y0, x0))
        best.sort(reverse=True)
        taken = 0
        for n, y0, x0 in best:
            if taken == per_view or n == 0:
                break
            crop = np.ascontiguousarray(rgb[y0:y0 + SZ, x0:x0 + SZ])
            _, _, lb = orc.slic(rgbx_of(crop), S, search=0)
            got = boundary_mask(lb)[inner]
            want = ref[y0:y0 + SZ, x0:x0 + SZ][inner]
            if not (got == full[y0:y0 + SZ, x0:x0 + SZ][inner]).all():
                continue  # SLIC not local enough here: the crop's interior differs from the full run
            taken += 1
            bad = int(np.count_nonzero(got != want))
            assert bad == n > 0
            print(f"residual crop green_new{k} @({y0},{x0}): {bad} of {want.size} interior pixels differ")
            out[f"rgb{i}"] = crop
            out[f"mask{i}"] = want
            out[f"meta{i}"] = np.array([0, y0, x0, MG, bad], np.int32)
            out[f"src{i}"] = np.array(f"green_new|{inp}|{ov}")
            i += 1
    np.savez_compressed(os.path.join(HERE, "ref_overlay_residual.npz"), n=np.int32(i), **out)
    print("wrote", os.path.join(HERE, "ref_overlay_residual.npz"))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "--residual":
    residual_crops()
