"""CPU suite: the C oracle against the independent numpy restatement
(tests/np_ref.py), the pinned math kernels against libm, and known answers.

No GPU needed.  Sizes keep the whole file to a few seconds.
"""
from __future__ import annotations

import math

import numpy as np
import pytest

import np_ref
import oracle.oracle as orc
from cases import CASES, PIXEL_CASES, build
from np_ref import (fma32, assign, boundary, cvt_f64, grid_labels, l8, ncc_volume, suppress, sweep_pixel_sad, update,
                    wta)


@pytest.fixture(scope="module", params=["c3x3_s8", "c2x2_s12", "c3x1_s16"])
def slic_case(request):
    c = CASES[request.param]
    b = build(c)
    return c, b


# ---------------------------------------------------------------- detmath ---
def test_detmath_exp_log_close_to_libm():
    xs = np.concatenate([np.linspace(-700, 700, 2001), np.linspace(-1, 1, 2001), [0.0, 1e-300, -1e-300]])
    for x in xs:
        e = orc.lib().orc_dm_exp
        e.restype = __import__("ctypes").c_double
        e.argtypes = [__import__("ctypes").c_double]
        ref = math.exp(x)
        got = e(x)
        assert abs(got - ref) <= 4e-16 * ref + 1e-320, (x, got, ref)
    lg = orc.lib().orc_dm_log
    lg.restype = __import__("ctypes").c_double
    lg.argtypes = [__import__("ctypes").c_double]
    for x in np.concatenate([np.geomspace(1e-300, 1e300, 1001), np.linspace(0.5, 2, 1001)]):
        assert abs(lg(x) - math.log(x)) <= 4e-16 * max(1.0, abs(math.log(x))), x


def test_detmath_powr_cube_root():
    import ctypes as C
    pw = orc.lib().orc_dm_powrf
    pw.restype = C.c_float
    pw.argtypes = [C.c_float, C.c_float]
    third = np.float32(1.0) / np.float32(3.0)
    for x in np.linspace(0.008857, 1.2, 997, dtype=np.float32):
        got = pw(float(x), float(third))
        ref = float(np.float32(float(x) ** float(third)))
        assert abs(got - ref) <= 2 * np.spacing(np.float32(ref)), (x, got, ref)
    assert pw(0.0, float(third)) == 0.0


def test_detmath_expf():
    import ctypes as C
    ef = orc.lib().orc_dm_expf
    ef.restype = C.c_float
    ef.argtypes = [C.c_float]
    for x in np.linspace(-80, 80, 4001, dtype=np.float32):
        ref = np.float32(math.exp(float(x)))
        got = np.float32(ef(float(x)))
        assert abs(float(got) - float(ref)) <= float(np.spacing(ref)), (x, got, ref)


# ------------------------------------------------------------- colour/grid ---
def test_cvt_known_answers():
    px = np.array([[[255, 255, 255, 0], [0, 0, 0, 0], [0, 0, 255, 0], [255, 0, 0, 0]]], np.uint8)
    lab = orc.cvt(px)
    assert abs(lab[0, 0, 0] - 100.0) < 0.01 and abs(lab[0, 0, 1]) < 0.05 and abs(lab[0, 0, 2]) < 0.05
    assert lab[0, 1, 0] == 0.0 and lab[0, 1, 1] == 0.0 and lab[0, 1, 2] == 0.0
    # R/B swap: s2 is RED in the reference's reading (rgb2lab(s0=B,...))
    assert abs(lab[0, 2, 0] - 53.24) < 0.05 and lab[0, 2, 1] > 75
    assert abs(lab[0, 3, 0] - 32.30) < 0.05 and lab[0, 3, 2] < -100


def test_cvt_matches_f64_model():
    rng = np.random.default_rng(3)
    px = rng.integers(0, 256, (37, 53, 4), dtype=np.uint8)
    lab = orc.cvt(px)
    ref = cvt_f64(px)
    np.testing.assert_allclose(lab[..., :3], ref, atol=2e-3)
    assert (lab[..., 3] == 0).all()


def test_l8_bit_exact():
    rng = np.random.default_rng(4)
    lab = np.zeros((31, 47, 4), np.float32)
    lab[..., 0] = rng.uniform(-5, 110, (31, 47)).astype(np.float32)
    lab[0, :4, 0] = [0.0, 99.99, 100.0, 100.0 / 2.55]
    assert np.array_equal(orc.l8(lab), l8(lab))


@pytest.mark.parametrize("W,H,S", [(100, 70, 8), (37, 29, 1), (250, 170, 40), (64, 64, 16)])
def test_grid_labels(W, H, S):
    _, sp, lb = orc.grid(np.zeros((H, W, 4), np.uint8), S)
    assert np.array_equal(lb, grid_labels(W, H, S))
    mw, mh = orc.map_size(W, H, S)
    assert sp.shape == (mh, mw, 8) and lb.max() < mw * mh


# ------------------------------------------------------------------- SLIC ---
def test_assign_bit_exact(slic_case):
    c, b = slic_case
    S = c["S"]
    lab = orc.cvt(b["stack"][0])
    sp = orc.init_centers(lab, S)
    assert np.array_equal(orc.assign(lab, sp, S), assign(lab, sp, S))


def test_update_bit_exact(slic_case):
    c, b = slic_case
    S = c["S"]
    lab = orc.cvt(b["stack"][1])
    lb = orc.assign(lab, orc.init_centers(lab, S), S)
    got = orc.update(lab, lb, S)
    ref = update(lab, lb, S)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_slic_pipeline_bit_exact(slic_case):
    """do_super_pixel_seg = init, assign, (update, assign) x no_iter."""
    c, b = slic_case
    S = c["S"]
    lab, sp, lb = orc.slic(b["stack"][0], S, no_iter=3)
    l2 = orc.cvt(b["stack"][0])
    s2 = orc.init_centers(l2, S)
    b2 = assign(l2, s2, S)
    for _ in range(3):
        s2 = update(l2, b2, S)
        b2 = assign(l2, s2, S)
    assert np.array_equal(lb, b2)
    assert np.array_equal(sp.view(np.uint32), s2.view(np.uint32))


def test_slic_invariants(slic_case):
    c, b = slic_case
    S, W, H = c["S"], c["W"], c["H"]
    _, sp, lb = orc.slic(b["stack"][0], S)
    mw, mh = orc.map_size(W, H, S)
    assert lb.max() < mw * mh
    # every pixel's label is one of the 2x2 candidate centres around its cell
    y, x = np.mgrid[0:H, 0:W]
    lx, ly = lb % mw, lb // mw
    assert (np.abs(lx.astype(int) - x // S) <= 1).all() and (np.abs(ly.astype(int) - y // S) <= 1).all()
    # ids, counts
    assert np.array_equal(sp[..., 0].reshape(-1), np.arange(mw * mh, dtype=np.float32))
    n = sp[..., 6]
    assert (n >= 0).all() and n.sum() <= W * H


def test_enforce_connectivity_bit_exact(slic_case):
    c, b = slic_case
    S = c["S"]
    _, _, lb0 = orc.slic(b["stack"][2 % b["V"]], S)
    _, _, lb1 = orc.slic(b["stack"][2 % b["V"]], S, enforce_connectivity=True)
    assert np.array_equal(lb1, suppress(suppress(lb0)))


# --------------------------------------------------------- sweep / boundary ---
def test_boundary_bit_exact(slic_case):
    c, b = slic_case
    S = c["S"]
    outs = [orc.slic(b["stack"][v], S) for v in range(b["V"])]
    sp = np.stack([o[1] for o in outs])
    lb = np.stack([o[2] for o in outs])
    assert np.array_equal(orc.boundary(sp, lb, S), boundary(sp, lb, S))


@pytest.mark.parametrize("name", list(PIXEL_CASES))
def test_sweep_pixel_sad_bit_exact(name):
    c = PIXEL_CASES[name]
    b = build(c)
    lab = orc.cvt(b["stack"])
    lv = b["levels"][:8]
    got = orc.sweep_pixel_sad(lab, lv, b["vs"], b["sn"], c["aw"], c["bl"])
    ref = sweep_pixel_sad(lab, lv, b["vs"], b["sn"], c["aw"], c["bl"])
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("name,K", [("c2x1_pix", 5), ("c2x2_pix", 5), ("c3x1_pix_odd", 7), ("c2x2_pix", 3)])
def test_ncc_volume_bit_exact(name, K):
    c = PIXEL_CASES[name]
    b = build(c)
    q = orc.l8(orc.cvt(b["stack"]))
    for z in range(b["V"]):
        got = orc.ncc_volume(q, b["levels"], b["vs"], b["sn"], c["aw"], c["bl"], K, z)
        ref = ncc_volume(q, b["levels"], b["vs"], b["sn"], c["aw"], c["bl"], K, z)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), z


def test_fma32_correctly_rounded():
    """np_ref.fma32 (the NCC restatement's fma) equals the exactly rounded
    a*b+c, including sums that land on a float32 rounding midpoint."""
    from fractions import Fraction
    rng = np.random.default_rng(3)
    a = rng.standard_normal(4000).astype(np.float32)
    b = rng.standard_normal(4000).astype(np.float32)
    c = rng.standard_normal(4000).astype(np.float32)
    # midpoint cases: c = -(a*b) rounded + a tiny remainder
    c[:1000] = (-(a[:1000].astype(np.float64) * b[:1000])).astype(np.float32)
    a[1000:1100] = np.float32(1 + 2 ** -12)
    b[1000:1100] = np.float32(1 + 2 ** -12)
    c[1000:1100] = np.float32(2 ** 20)
    got = fma32(a, b, c)
    for i in range(len(a)):
        exact = Fraction(float(a[i])) * Fraction(float(b[i])) + Fraction(float(c[i]))
        lo = np.float32(float(exact))
        cands = [lo, np.nextafter(lo, np.float32(np.inf)), np.nextafter(lo, np.float32(-np.inf))]
        errs = [abs(Fraction(float(t)) - exact) for t in cands]
        m = min(errs)
        best = [t for t, e in zip(cands, errs) if e == m]
        if len(best) > 1:  # tie: even mantissa
            best = [t for t in best if (t.view(np.uint32) & 1) == 0]
        assert got[i].view(np.uint32) == best[0].view(np.uint32), (i, a[i], b[i], c[i])


def test_ncc_cost_range_and_identity():
    """Costs lie in [0, 2]; a view matched against an identical neighbour at
    zero shift costs 1 - 1 = 0 wherever it is textured."""
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, (32, 40), dtype=np.uint8)
    q = np.stack([img, img])
    vs = np.array([[1, 0], [0, 0]], np.int32)
    sn = np.array([1, 1], np.int32)
    vol = orc.ncc_volume(q, np.array([0, 1, 2], np.float32), vs, sn, 2, 1.0, 5, 0)
    assert vol.min() >= -1e-6 and vol.max() <= 2  # E = x s_r may round to 1+ulp
    inner = vol[0, 2:-2, 2:-2]
    assert np.allclose(inner, 0, atol=1e-6)
    assert (vol[0, :2] == 2).all() and (vol[0, :, :2] == 2).all()


def test_wta_bit_exact_with_ties():
    rng = np.random.default_rng(9)
    vol = rng.integers(0, 6, (17, 23, 29)).astype(np.float32) * np.float32(0.25)
    vol[:, 0, 0] = 1e6  # all-invalid pixel keeps disparity 0
    lv = np.arange(17, dtype=np.float32) * 2 + 1
    d0, c0 = orc.wta(vol, lv)
    d1, c1 = wta(vol, lv)
    assert np.array_equal(d0, d1) and np.array_equal(c0, c1)
    assert d0[0, 0] == 0 and c0[0, 0] == 0


def test_sweep_recovers_planar_disparity():
    """End-to-end sanity of the oracle: NCC+WTA on a rendered fronto-parallel
    stack recovers most of the ground-truth disparity."""
    c = PIXEL_CASES["c2x1_pix"]
    b = build(c)
    q = orc.l8(orc.cvt(b["stack"]))
    vol = orc.ncc_volume(q, b["levels"], b["vs"], b["sn"], c["aw"], c["bl"], 5, 0)
    d, _ = orc.wta(vol, b["levels"])
    gt = b["gt"][0] if b["gt"].ndim == 3 else b["gt"]
    inner = (slice(4, -4), slice(int(c["dmax"]) + 4, -4))
    assert np.mean(np.abs(d[inner] - gt[inner]) <= 1) > 0.6


def _fused_wta_model(vol, levels, nw):
    """numpy model of the fused sweep's winner-take-all (ncc.hip, FUSE): wave w
    owns levels w, w+nw, ...; per pixel it folds (smallest cost, its level,
    second smallest cost) in level order with strict <; the waves are merged
    lexicographically for the best, and the smallest cost outside best +- 1 is
    per wave its second smallest when its best level lies in the window, else
    its smallest."""
    D = vol.shape[0]
    init = np.float32(1000000.0)
    shp = vol.shape[1:]
    v0 = np.full((nw,) + shp, init, np.float32)
    v1 = np.full((nw,) + shp, init, np.float32)
    i0 = np.full((nw,) + shp, -1, np.int64)
    for dl in range(D):
        w = dl % nw
        c = vol[dl]
        v1[w] = np.minimum(v1[w], np.maximum(v0[w], c))  # med3(v0, v1, c)
        take = c < v0[w]
        i0[w] = np.where(take, dl, i0[w])
        v0[w] = np.minimum(v0[w], c)
    bv, bi = v0[0].copy(), i0[0].copy()
    for w in range(1, nw):
        take = (v0[w] < bv) | ((v0[w] == bv) & (i0[w] >= 0) & (i0[w] < bi))
        bv, bi = np.where(take, v0[w], bv), np.where(take, i0[w], bi)
    c2 = np.full(shp, init, np.float32)
    for w in range(nw):
        inwin = (i0[w] >= bi - 1) & (i0[w] <= bi + 1)
        c2 = np.minimum(c2, np.where(inwin, v1[w], v0[w]))
    disp = np.where(bi >= 0, levels[np.maximum(bi, 0)], np.float32(0)).astype(np.float32)
    conf = np.where((bi < 0) | (c2 == init), np.float32(0), c2 - bv).astype(np.float32)
    return disp, conf


@pytest.mark.parametrize("D", [1, 2, 3, 5, 9, 33, 128])
@pytest.mark.parametrize("nw", [4, 8])
def test_fused_wta_fold_equals_top4(D, nw):
    """The fused kernel's per-wave fold + merge gives k_wta's top-4 answer
    (oracle orc.wta), ties included: costs drawn from a few values so that
    equal costs at many levels are common."""
    rng = np.random.default_rng(1000 * D + nw)
    vol = rng.choice(np.array([0.25, 0.5, 0.5, 1.0, 1.5, 2.0], np.float32), size=(D, 23, 37)).astype(np.float32)
    vol[:, :3, :] = 2.0  # invalid-window rows: cost 2 at every level
    levels = np.arange(D, dtype=np.float32) + np.float32(3)
    od, oc = orc.wta(vol, levels)
    fd, fc = _fused_wta_model(vol, levels, nw)
    assert np.array_equal(fd.view(np.uint32), od.view(np.uint32))
    assert np.array_equal(fc.view(np.uint32), oc.view(np.uint32))


@pytest.mark.parametrize("seed", [1, 2])
def test_edge_magnitude_bit_exact(seed):
    """orc_edge (edge_compute_alternative, clcode.cl:161-195) against the
    numpy restatement, image borders included."""
    rng = np.random.default_rng(seed)
    rgbx = rng.integers(0, 256, (23, 37, 4), dtype=np.uint8)
    lab = orc.cvt(rgbx)
    assert np.array_equal(orc.edge(lab).view(np.uint32), np_ref.edge(lab).view(np.uint32))


@pytest.mark.parametrize("S", [8, 12])
def test_slic_edge_modes(S):
    """apply_edge_values between init_cluster_centers and the first assignment
    (clSLIC.cpp:84-86): mode 1 overwrites Lab with the magnitude and moves no
    centre; mode 2 keeps Lab and moves each centre to its least-edge
    neighbour (numpy restatement)."""
    from cl_multiview_stereo_amd import synth
    stack, _ = synth.make_stack(70, 45, 1, 1, 0, 7, 1.0, S)
    lab0 = orc.cvt(stack[0])
    e = np_ref.edge(lab0)
    lab1, _, _ = orc.slic(stack[0], S, 0.6, 0, edge_enable=1)
    assert np.array_equal(lab1[..., 0], e) and np.array_equal(lab1[..., 1], e) and np.array_equal(lab1[..., 2], e)
    _, sp1, lb1 = orc.slic(stack[0], S, 0.6, 0, edge_enable=1)
    init = orc.init_centers(lab0, S)
    assert np.array_equal(sp1[..., :6], init[..., :6])  # no centre moves (edge_img never written)
    assert np.array_equal(lb1, orc.assign(lab1, init, S))
    lab2, sp2, lb2 = orc.slic(stack[0], S, 0.6, 0, edge_enable=2)
    assert np.array_equal(lab2, lab0)
    moved = np_ref.apply_edge(lab0, e, init)
    assert np.array_equal(sp2[..., :6], moved[..., :6])
    assert (moved[..., 1:3] != init[..., 1:3]).any()
    assert np.array_equal(lb2, orc.assign(lab0, moved, S))


def test_round_half_away_identity():
    """k_remove_incons_q's round_ha: roundf(v) == truncf(v + copysignf(0.49999997f, v))
    for every float.  Exhaustive over the positive floats below 2^23 (above, every
    float is an integer and both sides return v; negatives are symmetric)."""
    c = np.float32(np.frombuffer(np.uint32(0x3EFFFFFF).tobytes(), np.float32)[0])
    top = int(np.frombuffer(np.float32(2.0 ** 23).tobytes(), np.uint32)[0])
    step = 1 << 25
    for lo in range(0, top, step):
        v = np.arange(lo, min(lo + step, top), dtype=np.uint32).view(np.float32)
        t = np.trunc(v + c)
        r = np.trunc(v)
        r = r + (v - r >= np.float32(0.5)).astype(np.float32)  # roundf: half away from zero
        assert np.array_equal(t, r), lo
    big = np.float32([2.0 ** 23, 2.0 ** 23 + 1, 2.0 ** 24 + 2, 3.0e38, np.inf])
    assert np.array_equal(np.trunc(big + c), big)
    assert np.array_equal(np.trunc(-big - c), -big)
