"""GPU parity of the per-pixel SAD sweep (initial_depth_estimation_v2 at S=1
grid semantics, clcode.cl:972-1069: the reference's own cost) against the
oracle (orc_sweep_pixel_sad), at the BASELINE configurations' geometry and on
the edge cases of the band-staged kernel (k_sad_band): image borders, ragged
tiles, levels past the last chunk, vertical neighbours with fractional row
shifts (bl_ratio 1.0359), no neighbours, textureless ties.  Bar: bit-exact."""
from __future__ import annotations

import os

import numpy as np
import pytest
import torch

from cl_multiview_stereo_amd import params, synth
from cl_multiview_stereo_amd.engine import CameraArray
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def _cam(aw, ah, dmin, dmax, nh, nv, bl, inc=1):
    vs, sn = params.flatten_subsets(params.neighbour_lists(aw, ah, nh, nv))
    return CameraArray(aw, bl, params.disparity_levels(dmin, dmax, inc), vs, sn)


def _check(engine, stack, cam, z0=0, z1=None, tag=""):
    lab, _ = engine.cvt(torch.from_numpy(stack).cuda())
    V = stack.shape[0]
    z1 = V if z1 is None else z1
    got = engine.sweep_pixel_sad(lab, cam, z0, z1).cpu().numpy()
    want = orc.sweep_pixel_sad(lab.cpu().numpy(), cam.levels, cam.view_subset, cam.subset_num, cam.array_width,
                               cam.bl_ratio, z0, z1)
    bad = np.count_nonzero(got.view(np.uint32) != want.view(np.uint32))
    assert bad == 0, f"{tag}: {bad}/{got.size} disparities differ, first {np.argwhere(got != want)[:3].tolist()}"


@pytest.mark.parametrize("z", [0, 2])
def test_sad_c2_band(engine, z):
    """C2's array (5x1, 4 neighbours up to 4 views away, levels 0..127) on a
    full-width 1080p band of 40 rows."""
    stack, _ = synth.make_stack(1920, 40, 5, 1, 0, 127, 1.0, 0x5EED + 2)
    _check(engine, stack, _cam(5, 1, 0, 127, 4, 0, 1.0), z, z + 1, f"c2 band z{z}")


def test_sad_c2_full_height_bands(engine):
    """C2 itself (5 views 1920x1080, levels 0..127, the bench's stack): the
    GPU sweeps every whole view; the oracle recomputes three 62-row bands of
    each -- the top, the middle tile rows and the bottom rows of the 1080-row
    image -- from the band's Lab rows plus the window's 2-row margin (with
    horizontal-only neighbours a row's taps stay within rows y-2..y+2, so the
    band's inner rows are exactly the full image's)."""
    W, H, R = 1920, 1080, 2
    stack, _ = synth.make_stack(W, H, 5, 1, 0, 127, 1.0, 0x5EED + 2)  # = bench.py's C2 stack
    cam = _cam(5, 1, 0, 127, 4, 0, 1.0)
    lab, _ = engine.cvt(torch.from_numpy(stack).cuda())
    got = engine.sweep_pixel_sad(lab, cam, 0, 5).cpu().numpy()
    labh = lab.cpu().numpy()
    for y0 in (0, H // 2 - 31, H - 62):
        y1 = y0 + 62
        b0, b1 = max(0, y0 - R), min(H, y1 + R)
        want = orc.sweep_pixel_sad(np.ascontiguousarray(labh[:, b0:b1]), cam.levels, cam.view_subset, cam.subset_num,
                                   cam.array_width, cam.bl_ratio)[:, y0 - b0:y1 - b0]
        g = got[:, y0:y1]
        bad = np.count_nonzero(g.view(np.uint32) != want.view(np.uint32))
        assert bad == 0, f"rows {y0}..{y1 - 1}: {bad}/{g.size} disparities differ"


def test_sad_reference_defaults_geometry(engine):
    """The reference's own 3x3 array with bl_ratio 1.0359 (fractional vertical
    shifts, per-row truncation), levels 30..60, every view."""
    stack, _ = synth.make_stack(200, 70, 3, 3, 30, 60, 1.0359, 99)
    _check(engine, stack, _cam(3, 3, 30, 60, 1, 1, 1.0359), tag="3x3")


@pytest.mark.parametrize("W,H,D", [(61, 9, 1), (60, 8, 7), (121, 17, 9), (37, 29, 13), (250, 33, 40)])
def test_sad_ragged(engine, W, H, D):
    """Tile edges (60 x 8 tiles), level counts around the 8-level chunk."""
    stack, _ = synth.make_stack(W, H, 3, 1, 0, D - 1, 1.0, W * 7 + H)
    _check(engine, stack, _cam(3, 1, 0, D - 1, 2, 0, 1.0), tag=f"{W}x{H} D{D}")


def test_sad_level_step_and_offset(engine):
    stack, _ = synth.make_stack(130, 40, 4, 2, 3, 45, 1.0359, 5)
    _check(engine, stack, _cam(4, 2, 3, 45, 2, 1, 1.0359, inc=3), tag="inc3")


def test_sad_ties_and_no_neighbours(engine):
    """Flat patches (equal costs at many levels: the first minimum in level
    order must win across the waves' level subsets) and a view whose
    neighbour list is empty (disparity 0 everywhere)."""
    stack, _ = synth.make_stack(150, 40, 3, 1, 0, 23, 1.0, 8)
    stack[:, 5:30, 20:90, :3] = 90
    cam = _cam(3, 1, 0, 23, 1, 0, 1.0)
    cam.subset_num[0] = 0
    cam = CameraArray(cam.array_width, cam.bl_ratio, cam.levels, cam.view_subset, cam.subset_num)
    _check(engine, stack, cam, tag="ties")


# every instantiation on a geometry it can stage: (array, neighbours, bl).  An
# explicitly named band variant never falls back to the gather kernel
# (MVS_E_UNSUPPORTED instead), so each case runs the kernel it names.
_VARIANTS = {
    "sys8": (3, 3, 1, 1, 1.0359),    # 8-level chunks, fractional vertical shifts (row table)
    "sys8x2": (3, 1, 2, 0, 1.0),     # 16-level chunks (affine rows)
    "gather": (3, 3, 1, 1, 1.0359),
}


@pytest.mark.parametrize("kind", sorted(_VARIANTS))
def test_sad_kernel_variants(engine, kind, monkeypatch):
    """Every instantiation (MVS_SAD_KERNEL is read per call), on several tile
    columns and rows (bx0 > 0 and by0 > 0 bands)."""
    monkeypatch.setenv("MVS_SAD_KERNEL", kind)
    aw, ah, nh, nv, bl = _VARIANTS[kind]
    stack, _ = synth.make_stack(190, 50, aw, ah, 0, 20, bl, 12)
    _check(engine, stack, _cam(aw, ah, 0, 20, nh, nv, bl), tag=kind)
    assert os.environ["MVS_SAD_KERNEL"] == kind


@pytest.mark.parametrize("table", [False, True])
@pytest.mark.parametrize("aw,ah,nh,nv", [(3, 3, 1, 1), (5, 1, 4, 0), (4, 3, 2, 2)])
def test_sad_affine_rows(engine, monkeypatch, aw, ah, nh, nv, table):
    """The systolic kernel's affine band addressing (every row shift integral:
    bl_ratio 1, whole levels; 64- and 128-column bands) against the row-table
    path (MVS_SAD_AFF set) on the same geometry, vertical and diagonal
    neighbours included."""
    monkeypatch.setenv("MVS_SAD_KERNEL", "sys8")
    if table:
        monkeypatch.setenv("MVS_SAD_AFF", "0")
    stack, _ = synth.make_stack(200, 60, aw, ah, 0, 19, 1.0, 21 + aw)
    _check(engine, stack, _cam(aw, ah, 0, 19, nh, nv, 1.0), tag=f"aff {aw}x{ah} table={table}")


def test_sad_explicit_variant_does_not_fall_back(engine, monkeypatch):
    """sys8x2 cannot stage a neighbour 5 cameras away (16 levels x 5 px = 75
    columns of shift: a band wider than its 128 columns): named explicitly it
    fails loudly instead of running the gather kernel."""
    monkeypatch.setenv("MVS_SAD_KERNEL", "sys8x2")
    stack, _ = synth.make_stack(140, 50, 6, 1, 0, 20, 1.0, 12)
    lab, _ = engine.cvt(torch.from_numpy(stack).cuda())
    with pytest.raises(Exception, match="cannot stage"):
        engine.sweep_pixel_sad(lab, _cam(6, 1, 0, 20, 5, 0, 1.0), 0, 6)
