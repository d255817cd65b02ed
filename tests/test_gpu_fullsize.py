"""Full-size parity of the BASELINE configurations whose later stages were
checked only on crops before round 5 ("What's missing" 1):

* C3 -- 5 views 1920x1080, NCC 5x5 x 128 levels, SLIC S = 32, superpixel
  refinement (5 propagations, kernel_size 1080) + cross-view consistency
  filter -- through the product Pipeline exactly as `bench.py --config c3`
  runs it (fused sweep, superpixel chain on the side stream).  Labels, the
  superpixel seeds, the per-pixel NCC disparity and confidence of every view
  (the headline kernel, k_ncc_mfma, at full size), the refined and the
  filtered maps are compared bit for bit
  with the oracle's full-size run (clcode.cl:1076-1931 refinement,
  :1995-2101 projection + removal; pipeline.cpp:162-175 order).
* C5 -- 5 views 4096x3072, SLIC S = 40 (the incomplete 16x16-tile update
  window, clcode.cl:552-558 / clSLIC.cpp:313) and the superpixel sweep of all
  five views (clcode.cl:972-1069), bit for bit.  (C5's NCC 7x7 x 256 sweep is
  checked at full size on three row bands in test_gpu_ncc_configs.py.)

The oracle needs a few seconds of host time for each (OpenMP)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from cl_multiview_stereo_amd import params, synth
from cl_multiview_stereo_amd.pipeline import Pipeline
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _bits(a, b, what):
    a, b = np.asarray(a), np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    if a.dtype.kind == "f":
        a, b = a.view(np.uint32), b.view(np.uint32)
    bad = np.count_nonzero(a != b)
    assert bad == 0, f"{what}: {bad} of {a.size} elements differ from the oracle"


def _settings(S, aw, dmin, dmax, K, cost="ncc"):
    return params.Settings(spixl_size=S, array_width=aw, array_height=1, min_disp=dmin, max_disp=dmax, inc=1,
                           neib_hor=4, neib_ver=0, bl_ratio=1.0, window=K, cost=cost)


def _oracle_segment(stack, S, cam, aw):
    outs = [orc.slic(stack[v], S) for v in range(stack.shape[0])]
    lab = np.stack([o[0] for o in outs])
    sp = np.stack([o[1] for o in outs])
    lb = np.stack([o[2] for o in outs])
    rep = orc.boundary(sp, lb, S)
    sp = orc.sweep(lab, sp, rep, cam.levels, cam.view_subset, cam.subset_num, aw, 1.0, S)
    return lab, sp, lb, rep


@pytest.mark.parametrize("concurrent", [True, False])
def test_c3_full_size(engine, concurrent):
    W, H, aw, S = 1920, 1080, 5, 32
    st = _settings(S, aw, 0, 127, 5)
    stack, _ = synth.make_stack(W, H, aw, 1, 0, 127, 1.0, 0x5EED + 2)  # = bench.py --config c3
    p = Pipeline(engine, st, W, H, pixel_cost="ncc", refine=True, filt=True, concurrent=concurrent, fused=True)
    out = p.exe_pipeline(torch.from_numpy(stack).to(engine.device))
    torch.cuda.synchronize()
    lab, sp, lb, rep = _oracle_segment(stack, S, p.cam, aw)
    _bits(out.labels.cpu().numpy().view(np.uint32), lb, "SLIC labels (5 views, S = 32)")
    _bits(out.spixl.cpu().numpy(), sp, "superpixel seeds after the sweep")
    _bits(out.rep.cpu().numpy(), rep, "superpixel extents")
    # the per-pixel depth map (the headline's fused NCC 5x5 x 128 sweep + WTA,
    # k_ncc_mfma at 1920x1080, every reference view) and its confidence, against
    # the oracle's fused definition: orc_ncc_volume + orc_wta per view
    cam = p.cam
    q = orc.l8(lab)
    for z in range(aw):
        od, oc = orc.wta(orc.ncc_volume(q, cam.levels, cam.view_subset, cam.subset_num, aw, 1.0, 5, z), cam.levels)
        _bits(out.disp[z].cpu().numpy(), od, f"per-pixel NCC disparity, view {z}, 1920x1080")
        _bits(out.conf[z].cpu().numpy(), oc, f"per-pixel NCC confidence, view {z}, 1920x1080")
    ref = orc.refine(sp, lb, rep, p.cam.view_subset, p.cam.subset_num, aw, 1.0, S, kernel_size=st.kernel_size,
                     kernel_step=st.kernel_step)
    _bits(out.disp_refined.cpu().numpy(), ref["disp"], "refined (fused) disparity, 5 views 1920x1080")
    proj, filtered = orc.filt(ref["disp"], aw, 1.0, 1.0)
    _bits(out.disp_filtered.cpu().numpy(), filtered, "filtered disparity, 5 views 1920x1080")
    assert np.count_nonzero(filtered) > 0.3 * filtered.size  # the filter keeps a real share of the map


def test_c5_full_size_slic_and_superpixel_sweep(engine):
    W, H, aw, S = 4096, 3072, 5, 40
    st = _settings(S, aw, 0, 255, 7)
    stack, _ = synth.make_stack(W, H, aw, 1, 0, 255, 1.0, 0x5EED + 2)  # = bench.py --config c5
    p = Pipeline(engine, st, W, H, pixel_cost=None, refine=False, filt=False)
    out = p.exe_pipeline(torch.from_numpy(stack).to(engine.device))
    torch.cuda.synchronize()
    assert S % 16 != 0  # the k_update window walk (incomplete 16x16-tile window), not the tile kernels
    lab, sp, lb, rep = _oracle_segment(stack, S, p.cam, aw)
    _bits(out.lab.cpu().numpy(), lab, "Lab (5 views, 12 MP)")
    _bits(out.labels.cpu().numpy().view(np.uint32), lb, "SLIC labels (5 views, 4096x3072, S = 40)")
    _bits(out.rep.cpu().numpy(), rep, "superpixel extents")
    _bits(out.spixl.cpu().numpy(), sp, "superpixel centres + seeds after the sweep (all 5 views)")
    mw, mh = params.map_size(W, H, S) if hasattr(params, "map_size") else orc.map_size(W, H, S)
    assert sp.shape[:3] == (aw, mh, mw)
