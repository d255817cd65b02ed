"""GPU parity of the NCC sweep at the BASELINE configurations' own geometry,
and of every kernel instantiation, against the oracle (orc_ncc_volume /
orc_wta, oracle/mvs_oracle.c).

* C5 (5x1 array, NCC 7x7, levels 0..255, 4096 columns): the neighbours are
  horizontal, so a row band of the full-width image carries the full image's
  arithmetic; the full 4096x3072x256 volume (3.22 G cells, past 2^31) is then
  checked on bands at the top, middle and bottom against the oracle run on the
  band's rows (the band's rows R away from its cut edges equal the full image's).
* C4 (8x4 array, 5 nearest neighbours, 128 levels): vertical and diagonal
  neighbours, whose taller LDS bands select the narrower variants.
* Every (K, levels per wave, waves, band width, row parity, fused) variant,
  forced per call through mvs_set_ncc_variant.
Bar: bit-exact (costs, disparities, confidences)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from cl_multiview_stereo_amd import params, synth
from cl_multiview_stereo_amd.engine import CameraArray
from oracle import oracle as orc

pytestmark = pytest.mark.gpu


def bits(a):
    a = a.cpu().numpy() if hasattr(a, "cpu") else np.asarray(a)
    return np.ascontiguousarray(a).view(np.uint32)


def same(a, b, what):
    a, b = bits(a), bits(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    bad = np.count_nonzero(a != b)
    assert bad == 0, f"{what}: {bad}/{a.size} differ, first at {np.argwhere(a != b)[:3].tolist()}"


@pytest.fixture
def eng(engine):
    engine.set_ncc_variant()
    yield engine
    engine.set_ncc_variant()  # back to automatic for the other tests


def _array(aw, ah, dmin, dmax, nh=0, nv=0, knn=None, bl=1.0):
    levels = params.disparity_levels(dmin, dmax, 1)
    lists = params.nearest_neighbours(aw, ah, knn) if knn else params.neighbour_lists(aw, ah, nh, nv)
    vs, sn = params.flatten_subsets(lists)
    return CameraArray(aw, bl, levels, vs, sn)


def _check_view(eng, l8, box, cam, z, K, want_vol=None, rows=None):
    """GPU volume / WTA / fused sweep of reference view z against the oracle
    (rows: compare only these rows, the oracle having run on the same rows)."""
    l8h = l8.cpu().numpy()
    want = orc.ncc_volume(l8h, cam.levels, cam.view_subset, cam.subset_num, cam.array_width, cam.bl_ratio, K, z) \
        if want_vol is None else want_vol
    od, oc = orc.wta(want, cam.levels)
    vol = eng.ncc_volume(l8, box, cam, z, K)
    sl = slice(None) if rows is None else rows
    same(vol[:, sl], want[:, sl], f"volume z{z} K{K}")
    disp, conf = eng.wta(vol, eng.levels_dev(cam))
    same(disp[sl], od[sl], f"wta disp z{z}")
    same(conf[sl], oc[sl], f"wta conf z{z}")
    fd, fc = eng.ncc_wta(l8, box, cam, z, K)
    same(fd[sl], od[sl], f"fused disp z{z}")
    same(fc[sl], oc[sl], f"fused conf z{z}")
    del vol


def test_c5_band_full_width(eng):
    """C5's combination on a 64-row band of the full 4096-column image:
    NCC 7x7, 256 levels, horizontal neighbours up to 4 views away (shifts up
    to 1020 columns)."""
    stack, _ = synth.make_stack(4096, 64, 5, 1, 0, 255, 1.0, 0x5EED + 5)
    cam = _array(5, 1, 0, 255, nh=4)
    lab, l8 = eng.cvt(torch.from_numpy(stack).cuda())
    box = eng.box_stats(l8, 7)
    for z in (0, 2, 4):
        _check_view(eng, l8, box, cam, z, 7)
    seen = eng.ncc_last_variant()
    assert seen["K"] == 7 and seen["FUSE"] == 1


def test_c5_full_size_bands(eng):
    """The full C5 size (4096x3072, 256 levels: the volume has 3.22 G cells,
    indices past 2^31 from level 171 on) against the oracle on three row
    bands, every level of the band's rows."""
    W, H, K, R = 4096, 3072, 7, 3
    stack, _ = synth.make_stack(W, H, 5, 1, 0, 255, 1.0, 0x5EED + 5)
    cam = _array(5, 1, 0, 255, nh=4)
    lab, l8 = eng.cvt(torch.from_numpy(stack).cuda())
    del lab
    box = eng.box_stats(l8, K)
    z = 2
    vol = eng.ncc_volume(l8, box, cam, z, K)
    disp, conf = eng.wta(vol, eng.levels_dev(cam))
    fd, fc = eng.ncc_wta(l8, box, cam, z, K)
    torch.cuda.synchronize()
    same(fd, disp, "fused == two-pass disparity (full size)")
    same(fc, conf, "fused == two-pass confidence (full size)")
    l8h = l8.cpu().numpy()
    for y0, y1 in ((0, 64), (2000, 2064), (H - 64, H)):
        c0, c1 = max(0, y0 - R), min(H, y1 + R)  # crop whose rows y0..y1-1 see the full image's windows
        want = orc.ncc_volume(np.ascontiguousarray(l8h[:, c0:c1]), cam.levels, cam.view_subset, cam.subset_num,
                              5, 1.0, K, z)
        rows = slice(y0 - c0, y1 - c0)
        same(vol[:, y0:y1], want[:, rows], f"volume rows {y0}..{y1}")
        od, oc = orc.wta(want, cam.levels)
        same(disp[y0:y1], od[rows], f"disp rows {y0}..{y1}")
        same(conf[y0:y1], oc[rows], f"conf rows {y0}..{y1}")
        same(fd[y0:y1], od[rows], f"fused disp rows {y0}..{y1}")


@pytest.mark.parametrize("bl,nb", [(1.0, "1"), (1.0359, "1"), (1.0, "2"), (1.0359, "2")])
def test_c4_geometry(eng, bl, nb, monkeypatch):
    """C4's array (8x4, 5 nearest neighbours: horizontal, vertical and
    diagonal) at 128 levels on a cropped image.  The taller bands of the
    vertical neighbours must select the 2- and 1-level-per-wave variants the
    full-size C4 run uses, and all of them must match the oracle.  nb = "1"
    (the default, MVS_NCC_NB): 32-level chunks with single-buffered bands where the
    double-buffered ones miss two workgroups per CU; "2": the 16-level form."""
    monkeypatch.setenv("MVS_NCC_NB", nb)
    aw, ah, W, H = 8, 4, 256, 72
    stack, _ = synth.make_stack(W, H, aw, ah, 0, 127, bl, 0x5EED + 4)
    cam = _array(aw, ah, 0, 127, knn=5, bl=bl)
    lab, l8 = eng.cvt(torch.from_numpy(stack).cuda())
    l8h = l8.cpu().numpy()
    box = eng.box_stats(l8, 5)
    variants = set()
    for z in range(aw * ah):
        want = orc.ncc_volume(l8h, cam.levels, cam.view_subset, cam.subset_num, aw, bl, 5, z)
        od, oc = orc.wta(want, cam.levels)
        vol = eng.ncc_volume(l8, box, cam, z, 5)
        v = eng.ncc_last_variant()
        variants.add((v["DPW"], v["NW"], v["BW"], v["PAR"], v["NB"]))
        same(vol, want, f"volume z{z}")
        d, c = eng.wta(vol, eng.levels_dev(cam))
        same(d, od, f"disp z{z}")
        same(c, oc, f"conf z{z}")
        fd, fc = eng.ncc_wta(l8, box, cam, z, 5)
        same(fd, od, f"fused disp z{z}")
        same(fc, oc, f"fused conf z{z}")
    dpws = {v[0] for v in variants}
    if nb == "1":  # every list but the corner views' (a neighbour two rows away) takes 32-level chunks
        assert 4 in dpws, f"single-buffered 32-level chunks expected, saw {sorted(variants)}"
        # the single-buffered kernel ran, seen directly (NB slot), for the mixed-parity 5-NN lists
        assert any(v[4] == 1 for v in variants), f"single-buffered bands expected, saw {sorted(variants)}"
    else:
        assert dpws & {1, 2}, f"C4 geometry should need a narrower variant, saw {sorted(variants)}"
        assert {v[4] for v in variants} == {2}, f"MVS_NCC_NB=2 must keep double buffers, saw {sorted(variants)}"


@pytest.mark.parametrize("form", ["auto", "22", "21", "12", "11"])
@pytest.mark.parametrize("bl,dmax,H", [(1.0, 127, 72), (1.0359, 99, 69)])
def test_mfma_vertical_forms(eng, form, bl, dmax, H, monkeypatch):
    """The matrix-core fused sweep for lists with vertical / diagonal
    neighbours (k_ncc_mfma<..., VERT>: C4's 8x4 array, 5 nearest neighbours),
    every view of the array, each (16-level blocks per chunk, band buffers)
    form forced through MVS_NCC_MFMA_V ("auto", MVS_NCC_MFMA_V=1 or unset:
    the launcher's choice under two workgroups per CU, the default; 0: the
    scalar kernels).  D = 128 (whole chunks) and D = 100 (dummy levels
    in the last chunk); bl = 1.0359: fractional vertical shifts, so a chunk's
    levels start on odd and even band rows; H = 69: an odd height (the dummy
    row of the pair planes) and a partial last tile row."""
    monkeypatch.setenv("MVS_NCC_MFMA_V", "1" if form == "auto" else form)
    aw, ah, W = 8, 4, 200
    stack, _ = synth.make_stack(W, H, aw, ah, 0, dmax, bl, 0x5EED + 6)
    cam = _array(aw, ah, 0, dmax, knn=5, bl=bl)
    lab, l8 = eng.cvt(torch.from_numpy(stack).cuda())
    l8h = l8.cpu().numpy()
    box = eng.box_stats(l8, 5)
    forms = []
    for z in range(aw * ah):
        want = orc.ncc_volume(l8h, cam.levels, cam.view_subset, cam.subset_num, aw, bl, 5, z)
        od, oc = orc.wta(want, cam.levels)
        fd, fc = eng.ncc_wta(l8, box, cam, z, 5)
        v = eng.ncc_last_variant()
        same(fd, od, f"fused disp z{z} form {form}")
        same(fc, oc, f"fused conf z{z} form {form}")
        if v["DPW"] >= 16:  # the matrix-core form ran
            assert v["PAR"] == 0 and v["FUSE"] == 1, v
            forms.append(f"{v['DPW'] // 16}{v['NB']}")
    # the corner views' lists hold a neighbour two rows away: their bands may
    # miss the LDS cap (80 KB auto, 160 KB forced) and take the scalar kernel
    # (at D = 100 the tail kernels' 128-column pitch: the 32-level
    # double-buffered bands miss 160 KB for every list)
    if form == "auto" or form != "22" or dmax == 127:
        assert len(forms) >= aw * ah - 4, forms
    if form != "auto":
        assert set(forms) <= {form}, forms


_VARIANTS = [(8, 4), (8, 2), (4, 4), (4, 2), (4, 1)]  # (waves, levels per wave): every instantiation
_BANDS = (64, 80, 96, 128, 192, 256)  # band pitch templates (columns per pair row)


@pytest.mark.parametrize("K", [5, 7])
@pytest.mark.parametrize("geom", ["horizontal", "vertical", "vertical_only"])
def test_every_ncc_variant(eng, K, geom):
    """Force each (waves, levels per wave) x band width x row-parity variant,
    plain and fused, and compare with the oracle; the launch must report the
    forced variant (a band width below what the shifts need rises to the
    smallest pitch that holds them: 128 horizontal, 80 for one column of
    shift range, 64 for vertical neighbours only)."""
    if geom == "horizontal":  # every band row starts on a pair: the EVEN kernel is eligible
        aw, ah, nh, nv, bl, W, H, dmax = 4, 1, 2, 0, 1.0, 150, 40, 39
    elif geom == "vertical":  # vertical neighbours with fractional shifts: odd band-row starts.  Few
        # levels, so that even the 32-level chunk's band at 256 columns fits the 160 KB LDS
        aw, ah, nh, nv, bl, W, H, dmax = 2, 3, 1, 1, 1.0359, 120, 56, 4
    else:  # a 1 x 3 column of cameras: no column shift at all
        aw, ah, nh, nv, bl, W, H, dmax = 1, 3, 0, 1, 1.0359, 100, 56, 4
    stack, _ = synth.make_stack(W, H, aw, ah, 0, dmax, bl, 77 + K)
    cam = _array(aw, ah, 0, dmax, nh=nh, nv=nv, bl=bl)
    lab, l8 = eng.cvt(torch.from_numpy(stack).cuda())
    l8h = l8.cpu().numpy()
    box = eng.box_stats(l8, K)
    z = 1
    want = orc.ncc_volume(l8h, cam.levels, cam.view_subset, cam.subset_num, aw, bl, K, z)
    od, oc = orc.wta(want, cam.levels)
    evens, seen = set(), set()
    dxs = [int(v) % aw - z % aw for v in cam.view_subset[z, :int(cam.subset_num[z])]]
    for nw, dpw in _VARIANTS:
        dc = nw * dpw  # columns of shift range in a chunk of dc whole levels: |dx| (dc' - 1)
        need = 64 + max(abs(dx) for dx in dxs) * (min(dc, dmax + 1) - 1)
        need = min(b for b in _BANDS if b >= need)
        for bw in _BANDS:
            for general in (False, True):
                eng.set_ncc_variant(nw, dpw, bw, general)
                tag = f"K{K} nw{nw} dpw{dpw} bw{bw} general{int(general)}"
                vol = eng.ncc_volume(l8, box, cam, z, K)
                v = eng.ncc_last_variant()
                assert (v["K"], v["NW"], v["DPW"], v["FUSE"]) == (K, nw, dpw, 0), (tag, v)
                assert v["BW"] == max(bw, need), (tag, v)
                seen.add(v["BW"])
                if general:
                    assert v["PAR"] == 0, (tag, v)
                evens.add(v["PAR"])
                same(vol, want, f"volume {tag}")
                fd, fc = eng.ncc_wta(l8, box, cam, z, K)
                v = eng.ncc_last_variant()
                assert (v["NW"], v["DPW"], v["BW"], v["FUSE"]) == (nw, dpw, max(bw, need), 1), (tag, v)
                same(fd, od, f"fused disp {tag}")
                same(fc, oc, f"fused conf {tag}")
    # every pitch from the narrowest the geometry allows (4-level chunks) up
    assert seen == {b for b in _BANDS if b >= {"horizontal": 80, "vertical": 80, "vertical_only": 64}[geom]}, seen
    # row-parity mode (kParMixed 0 / kParEven 1 / kParOdd 2): K = 5 horizontal
    # bands start on a row pair (R + tymax even), K = 7 (R = 3) horizontal
    # bands on an odd row; fractional vertical shifts mix both
    assert evens == ({0, 1 if K == 5 else 2} if geom == "horizontal" else {0})


@pytest.mark.parametrize("case", ["c2_like", "c4_like", "c5_like", "frac_vertical", "forced"])
def test_ncc_wta_range(eng, case):
    """mvs_ncc_wta_range_d: runs of reference views per launch (one kernel
    boundary per run, up to 8 views, the run's widest band stride and parity)
    equal the per-view fused sweep and the oracle, bit for bit -- views with
    different band widths (C2: 128 vs 192), different variants inside one call
    (C4: 2- and 1-level-per-wave runs), more views than one launch holds, a
    sub-range, and a forced variant."""
    K, z0, z1 = 5, None, None
    if case == "c2_like":
        aw, ah, W, H, dmax, nh, nv, knn, bl = 5, 1, 200, 40, 127, 4, 0, None, 1.0
    elif case == "c4_like":
        aw, ah, W, H, dmax, nh, nv, knn, bl = 8, 4, 200, 48, 127, 0, 0, 5, 1.0
    elif case == "c5_like":
        aw, ah, W, H, dmax, nh, nv, knn, bl, K = 5, 1, 300, 30, 100, 4, 0, None, 1.0, 7
        z0, z1 = 1, 4
    elif case == "frac_vertical":
        aw, ah, W, H, dmax, nh, nv, knn, bl = 3, 3, 96, 60, 20, 1, 1, None, 1.0359
    else:
        aw, ah, W, H, dmax, nh, nv, knn, bl = 4, 2, 120, 40, 39, 1, 1, None, 1.0
        eng.set_ncc_variant(4, 2, 192, False)
    V = aw * ah
    z0 = 0 if z0 is None else z0
    z1 = V if z1 is None else z1
    stack, _ = synth.make_stack(W, H, aw, ah, 0, dmax, bl, 0x5EED + 9)
    cam = _array(aw, ah, 0, dmax, nh=nh, nv=nv, knn=knn, bl=bl)
    lab, l8 = eng.cvt(torch.from_numpy(stack).cuda())
    box = eng.box_stats(l8, K)
    rd, rc = eng.ncc_wta_range(l8, box, cam, z0, z1, K)
    l8h = l8.cpu().numpy()
    for i, z in enumerate(range(z0, z1)):
        fd, fc = eng.ncc_wta(l8, box, cam, z, K)
        same(rd[i], fd, f"range vs per-view disp z{z}")
        same(rc[i], fc, f"range vs per-view conf z{z}")
        if i % 3 == 0:
            want = orc.ncc_volume(l8h, cam.levels, cam.view_subset, cam.subset_num, aw, bl, K, z)
            od, oc = orc.wta(want, cam.levels)
            same(rd[i], od, f"range vs oracle disp z{z}")
            same(rc[i], oc, f"range vs oracle conf z{z}")
    # no confidence requested
    nd, _ = eng.ncc_wta_range(l8, box, cam, z0, z1, K, want_conf=False)
    same(nd, rd, "range without confidence")


@pytest.mark.parametrize("bl", [1.0, 1.0359])
def test_sweep_spixl_transposed_vertical(engine, monkeypatch, bl):
    """The superpixel sweep reads vertical neighbours (same camera column) from
    a transposed copy of their Lab and diagonal ones from sheared copies: C4's
    array (5 nearest neighbours: vertical, horizontal, diagonal) at 128
    levels, every reference view, equal to the row-major gathers
    (MVS_SWEEP_TRANSPOSE=0) and to the oracle; also a view sub-range."""
    aw, ah, W, H, S = 8, 4, 160, 96, 16
    stack, _ = synth.make_stack(W, H, aw, ah, 0, 127, bl, 0x5EED + 11)
    cam = _array(aw, ah, 0, 127, knn=5, bl=bl)
    lab, _ = engine.cvt(torch.from_numpy(stack).cuda())
    sp, lb = engine.slic(lab, S)
    rep = engine.boundary(sp, lb, S)
    out = {}
    for mode in ("0", "1", "2"):  # row-major only / + transposed vertical / + sheared diagonal
        monkeypatch.setenv("MVS_SWEEP_TRANSPOSE", mode)
        s = sp.clone()
        engine.sweep_spixl(lab, s, rep, cam, S)
        out[mode] = s
    same(out["1"], out["0"], "transposed vs row-major superpixel sweep")
    same(out["2"], out["0"], "transposed + sheared vs row-major superpixel sweep")
    osp = orc.sweep(lab.cpu().numpy(), sp.cpu().numpy(), rep.cpu().numpy(), cam.levels, cam.view_subset,
                    cam.subset_num, aw, bl, S)
    same(out["2"][..., 7], osp[..., 7], "re-laid superpixel sweep vs oracle")
    monkeypatch.delenv("MVS_SWEEP_TRANSPOSE")
    s = sp.clone()
    engine.sweep_spixl(lab, s, rep, cam, S, 12, 16)
    same(s[12:16], out["2"][12:16], "view sub-range")


def _box_planes_np(l8: np.ndarray, K: int):
    """numpy restatement of the window planes (include/mvs.h layout): per
    (view, row pair, column) the floats {a(y), a(y+1), b(y), b(y+1)} with
    a = K^2 / sqrt(var), b = (S - 128 K^2) / sqrt(var) (NaN where the window
    leaves the image, 0 where var == 0), and the 8 bytes from column x - R of
    each row as int8 (q ^ 0x80; the dummy row H of an odd height and columns
    outside the image as 0 ^ 0x80, the dummy row's 8 bytes as 0)."""
    V, H, W = l8.shape
    R, NK = K // 2, K * K
    Hp = H + (H & 1)
    pad = np.zeros((V, Hp + 2 * R, W + 8 + R), np.int64)
    pad[:, R:R + H, R:R + W] = l8
    s = np.zeros((V, Hp, W), np.int64)
    ss = np.zeros((V, Hp, W), np.int64)
    for j in range(K):
        for i in range(K):
            v = pad[:, j:j + Hp, i:i + W]
            s += v
            ss += v * v
    var = (NK * ss - s * s).astype(np.int32)
    y = np.arange(Hp)[None, :, None]
    x = np.arange(W)[None, None, :]
    valid = (x - R >= 0) & (x + R < W) & (y - R >= 0) & (y + R < H)
    with np.errstate(divide="ignore", invalid="ignore"):
        sv = np.where(var != 0, np.float32(1) / np.sqrt(var.astype(np.float32)), np.float32(0)).astype(np.float32)
    sv = np.where(valid, sv, np.float32(np.nan)).astype(np.float32)
    av = (np.float32(NK) * sv).astype(np.float32)
    bv = ((s - 128 * NK).astype(np.float32) * sv).astype(np.float32)
    st = np.empty((V, Hp // 2, W, 4), np.float32)
    st[..., 0], st[..., 1], st[..., 2], st[..., 3] = av[:, 0::2], av[:, 1::2], bv[:, 0::2], bv[:, 1::2]
    rows = np.stack([pad[:, R:R + Hp, k:k + W] for k in range(8)], -1).astype(np.uint8) ^ 0x80  # column x - R + k
    rows[:, H:] = 0
    pk = rows.reshape(V, Hp // 2, 2, W, 8).transpose(0, 1, 3, 2, 4).reshape(V, Hp // 2, W, 16)
    return st, pk


@pytest.mark.parametrize("K", [5, 7])
@pytest.mark.parametrize("W,H", [(160, 37), (150, 40), (67, 21), (64, 16)])
def test_box_planes(engine, K, W, H):
    """k_box_stats against a numpy restatement, bit-exact: widths on and off
    4-byte rows (the dword and byte tile fills), odd heights (the dummy row),
    partial 64-column tiles."""
    rng = np.random.default_rng(W * 1000 + H + K)
    l8 = rng.integers(0, 256, (3, H, W), dtype=np.uint8)
    l8[1, :, : W // 2] = 77  # flat windows: var == 0
    box = engine.box_stats(torch.from_numpy(l8).cuda(), K).cpu().numpy()
    Hp = H + (H & 1)
    st, pk = _box_planes_np(l8, K)
    got_st = box[0].reshape(-1).view(np.float32).reshape(3, Hp // 2, W, 4)
    got_pk = box[1].reshape(-1).view(np.uint8).reshape(3, Hp // 2, W, 16)
    same(got_st, st, f"stats K{K} {W}x{H}")
    assert np.array_equal(got_pk, pk), f"packed rows K{K} {W}x{H}"


@pytest.mark.parametrize("D,nn", [(1600, 16), (4000, 16)])
def test_fused_large_d_horizontal(eng, D, nn):
    """A horizontal list whose matrix-core run would not fit the LDS (ADVICE
    r05): 16 horizontal neighbours (a 17x1 array, 8 views either side) and
    fractional levels 0.05 apart, so every 32-level chunk's band stays within
    the 192-column pitch.  k_ncc_mfma keeps a run's level offsets in LDS
    (chunks x neighbours x 64 B): at D = 1600 they fit and the matrix-core
    form runs (DPW >= 16 in the report); at D = 4000 (128 KB of offsets beside
    the 128-column bands) they would pass 160 KB and the scalar fused kernel
    takes the view.  Both bit-exact against the oracle."""
    aw, W, H, z = 17, 72, 12, 8
    levels = (np.arange(D, dtype=np.float32) * np.float32(0.05)).astype(np.float32)
    vs, sn = params.flatten_subsets(params.neighbour_lists(aw, 1, nn // 2, 0))
    cam = CameraArray(aw, 1.0, levels, vs, sn)
    assert int(cam.subset_num[z]) == nn
    stack, _ = synth.make_stack(W, H, aw, 1, 0, 3, 1.0, 0xD0 + D)
    lab, l8 = eng.cvt(torch.from_numpy(stack).cuda())
    box = eng.box_stats(l8, 5)
    want = orc.ncc_volume(l8.cpu().numpy(), cam.levels, cam.view_subset, cam.subset_num, aw, 1.0, 5, z)
    od, oc = orc.wta(want, cam.levels)
    fd, fc = eng.ncc_wta(l8, box, cam, z, 5)
    v = eng.ncc_last_variant()
    assert v["FUSE"] == 1 and (v["DPW"] >= 16) == (D == 1600), v  # DPW >= 16: the matrix-core form
    same(fd, od, f"fused disp D{D}")
    same(fc, oc, f"fused conf D{D}")


@pytest.mark.parametrize("W,H,dmax,aw,nh", [(150, 27, 63, 5, 4), (130, 40, 100, 5, 4), (64, 8, 15, 3, 1),
                                            (200, 33, 40, 7, 3), (97, 19, 31, 4, 2)])
def test_mfma_k7(eng, monkeypatch, W, H, dmax, aw, nh):
    """The matrix-core K = 7 fused sweep (k_ncc_mfma<7, ...>: 2 x 8-pixel
    blocks, two MFMAs per level block over the 16-row footprint, 16-level
    chunks) on horizontal lists: ragged tiles (W, H off the 64 x 8 tile, odd H),
    image borders, whole and partial last chunks (D = 16, 64 / D = 101, 41, 32),
    shifts up to 4 columns per level (band pitch 128, 192 with a tail), the
    triple-buffered form and the double-buffered one (MVS_NCC_MFMA7_NB=2).
    Every reference view against the oracle and against the scalar fused
    kernel (MVS_NCC_MFMA7=0), bit for bit."""
    stack, _ = synth.make_stack(W, H, aw, 1, 0, dmax, 1.0, 0x7A + W + H)
    cam = _array(aw, 1, 0, dmax, nh=nh)
    lab, l8 = eng.cvt(torch.from_numpy(stack).cuda())
    box = eng.box_stats(l8, 7)
    l8h = l8.cpu().numpy()
    for z in range(aw):
        want = orc.ncc_volume(l8h, cam.levels, cam.view_subset, cam.subset_num, aw, 1.0, 7, z)
        od, oc = orc.wta(want, cam.levels)
        monkeypatch.delenv("MVS_NCC_MFMA7", raising=False)
        fd, fc = eng.ncc_wta(l8, box, cam, z, 7)
        v = eng.ncc_last_variant()
        assert (v["K"], v["DPW"], v["FUSE"]) == (7, 16, 1), v  # DPW 16: the matrix-core form, 16-level chunks
        same(fd, od, f"k7 mfma disp z{z}")
        same(fc, oc, f"k7 mfma conf z{z}")
        # the 128-column pitch without a partial chunk also has a triple-
        # buffered form (bands two steps ahead, counted vmcnt before each
        # barrier; MVS_NCC_MFMA7_NB picks it): the other form, the same bits
        tail = (dmax + 1) % 16 != 0
        if not tail and v["BW"] == 128:
            other = 2 if v["NB"] == 3 else 3
            monkeypatch.setenv("MVS_NCC_MFMA7_NB", str(other))
            d2, c2 = eng.ncc_wta(l8, box, cam, z, 7)
            assert eng.ncc_last_variant()["NB"] == other
            same(d2, fd, f"k7 mfma double- vs triple-buffered disp z{z}")
            same(c2, fc, f"k7 mfma double- vs triple-buffered conf z{z}")
            monkeypatch.delenv("MVS_NCC_MFMA7_NB")
        monkeypatch.setenv("MVS_NCC_MFMA7", "0")
        sd, sc = eng.ncc_wta(l8, box, cam, z, 7)
        assert eng.ncc_last_variant()["DPW"] < 16
        same(sd, fd, f"k7 scalar vs mfma disp z{z}")
        same(sc, fc, f"k7 scalar vs mfma conf z{z}")


@pytest.mark.parametrize("geom", ["c4_knn5", "horizontal_forced"])
def test_scalar_band_dma_forms(eng, monkeypatch, geom):
    """The scalar kernels' band staging: buffer descriptors with the pair row
    as the scalar offset (the default for view planes under 2 GB) against the
    64-bit per-lane addresses (MVS_NCC_PLANE32=0), both against the oracle:
    C4's 5-NN lists (tall single-buffered vertical / diagonal bands, the
    corner views' 2-level form, a fractional vertical shift) and a horizontal
    list on a forced scalar variant (double-buffered bands); fused sweep and
    cost volume, bit for bit."""
    if geom == "c4_knn5":
        aw, ah, W, H, dmax, bl, zs = 8, 4, 136, 45, 127, 1.0359, (0, 5, 13, 31)
        cam = _array(aw, ah, 0, dmax, knn=5, bl=bl)
    else:
        aw, ah, W, H, dmax, bl, zs = 5, 1, 150, 27, 63, 1.0, (0, 2)
        cam = _array(aw, ah, 0, dmax, nh=4)
        eng.set_ncc_variant(8, 4, 192, False)
    stack, _ = synth.make_stack(W, H, aw, ah, 0, dmax, bl, 0xB0F + W)
    lab, l8 = eng.cvt(torch.from_numpy(stack).cuda())
    box = eng.box_stats(l8, 5)
    l8h = l8.cpu().numpy()
    monkeypatch.setenv("MVS_NCC_MFMA_V", "0")  # the scalar kernels for the vertical lists too
    for z in zs:
        want = orc.ncc_volume(l8h, cam.levels, cam.view_subset, cam.subset_num, aw, bl, 5, z)
        od, oc = orc.wta(want, cam.levels)
        for form in ("1", "0"):
            monkeypatch.setenv("MVS_NCC_PLANE32", form)
            fd, fc = eng.ncc_wta(l8, box, cam, z, 5)
            assert eng.ncc_last_variant()["DPW"] < 16  # a scalar kernel
            same(fd, od, f"fused disp z{z} plane32={form}")
            same(fc, oc, f"fused conf z{z} plane32={form}")
            vol = eng.ncc_volume(l8, box, cam, z, 5)
            same(vol, want, f"volume z{z} plane32={form}")
        monkeypatch.delenv("MVS_NCC_PLANE32")
