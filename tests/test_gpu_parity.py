"""GPU parity: the HIP path (libmvs.so through the C-ABI) against the CPU
oracle (oracle/mvs_oracle.c) on the same seeded inputs.

Bar: bit-exact for every stage -- labels, extents, disparities (integer-valued
levels), Lab, superpixel statistics, NCC costs and refinement states -- because
both sides evaluate the same pinned numerical definition (include/mvs_detmath.h,
IEEE ops, no contraction).  Parity against the reference's own execution is
UNPINNED (see oracle/mvs_oracle.c header and DESIGN.md).
"""
import numpy as np
import pytest
import torch

from cl_multiview_stereo_amd import params, synth
from cl_multiview_stereo_amd.engine import CameraArray
from oracle import oracle as orc
from tests.cases import CASES, PIXEL_CASES, as_u32, build

pytestmark = pytest.mark.gpu


def dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def assert_bits(a, b, what):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape, (what, a.shape, b.shape)
    if a.dtype.kind == "f":
        eq = a.view(np.uint32 if a.dtype == np.float32 else np.uint64) == b.view(
            np.uint32 if b.dtype == np.float32 else np.uint64)
    else:
        eq = a == b
    bad = np.count_nonzero(~eq)
    if bad:
        idx = np.argwhere(~eq)[:5]
        pytest.fail(f"{what}: {bad}/{a.size} elements differ; first at {idx.tolist()}: "
                    f"{[a[tuple(i)] for i in idx]} vs {[b[tuple(i)] for i in idx]}")


# ---------------------------------------------------------------------------
def test_cvt_all_colours(engine):
    # every (r, g, b) on a 4-step lattice plus the extremes, R/B swap included
    v = np.arange(0, 256, 4, dtype=np.uint8)
    r, g, b = np.meshgrid(v, v, v, indexing="ij")
    rgbx = np.stack([r.ravel(), g.ravel(), b.ravel(), np.zeros(r.size, np.uint8)], -1)
    rgbx = np.concatenate([rgbx, np.array([[255, 255, 255, 0], [0, 0, 0, 0], [255, 0, 0, 0]], np.uint8)])
    W = 512
    H = (len(rgbx) + W - 1) // W
    pad = np.zeros((H * W - len(rgbx), 4), np.uint8)
    img = np.concatenate([rgbx, pad]).reshape(1, H, W, 4)
    lab, l8 = engine.cvt(dev(img))
    want = orc.cvt(img[0])
    assert_bits(lab.cpu().numpy()[0], want, "lab")
    assert_bits(l8.cpu().numpy()[0], orc.l8(want), "l8")


@pytest.mark.parametrize("name", list(CASES))
def test_slic(engine, name):
    c = CASES[name]
    b = build(c)
    conn = name == "c2x2_s12"
    lab, _ = engine.cvt(dev(b["stack"]))
    sp, lb = engine.slic(lab, c["S"], 0.6, 5, conn)
    sp, lb, lab = sp.cpu().numpy(), as_u32(lb), lab.cpu().numpy()
    for v in range(b["V"]):
        olab, osp, olb = orc.slic(b["stack"][v], c["S"], 0.6, 5, conn)
        assert_bits(lab[v], olab, f"lab v{v}")
        assert_bits(lb[v], olb, f"labels v{v}")
        assert_bits(sp[v][..., :7], osp[..., :7], f"spixl v{v}")


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("name", ["c3x1_s8", "c5x1_s32", "c2x1_s40"])
def test_slic_edge(engine, name, mode):
    """apply_edge_values (clSLIC.cpp:84-86, 186-233; clcode.cl:161-248):
    mode 1 = the reference's path as it behaves (Lab overwritten in place by
    the edge magnitude, no centre moved), mode 2 = the intended perturbation.
    Lab, labels and centres bit-exact vs the oracle, both assignment paths."""
    c = CASES[name]
    b = build(c)
    lab, _ = engine.cvt(dev(b["stack"]))
    sp, lb = engine.slic(lab, c["S"], 0.6, 5, edge_enable=mode)
    sp, lb, lab = sp.cpu().numpy(), as_u32(lb), lab.cpu().numpy()
    for v in range(b["V"]):
        olab, osp, olb = orc.slic(b["stack"][v], c["S"], 0.6, 5, edge_enable=mode)
        assert_bits(lab[v], olab, f"lab v{v}")
        assert_bits(lb[v], olb, f"labels v{v}")
        assert_bits(sp[v][..., :7], osp[..., :7], f"spixl v{v}")


@pytest.mark.parametrize("no_iter", [0, 5])
@pytest.mark.parametrize("name", ["c3x1_s8", "c5x1_s32", "c2x1_s40", "c2x2_s12"])
def test_slic_search3x3(engine, name, no_iter):
    """mvs_slic_params.search = 1: the 3x3 candidate loop behind the
    reference's comment switch (clcode.cl:496-516), with which the reference's
    kept depth outputs were produced.  Both assignment
    paths (k_assign for S % 16 != 0, k_assign_tiles for S = 32)."""
    c = CASES[name]
    b = build(c)
    lab, _ = engine.cvt(dev(b["stack"]))
    sp, lb = engine.slic(lab, c["S"], 0.6, no_iter, search=1)
    sp, lb = sp.cpu().numpy(), as_u32(lb)
    for v in range(b["V"]):
        _, osp, olb = orc.slic(b["stack"][v], c["S"], 0.6, no_iter, search=1)
        assert_bits(lb[v], olb, f"labels v{v}")
        assert_bits(sp[v][..., :7], osp[..., :7], f"spixl v{v}")


@pytest.mark.parametrize("name", ["c3x1_s8", "c5x1_s32"])
def test_slic_each_pass(engine, name):
    """Per-pass parity of the assign/update loop (no_iter = 0, 1, 2)."""
    c = CASES[name]
    b = build(c)
    lab, _ = engine.cvt(dev(b["stack"][:1]))
    for it in range(3):
        sp, lb = engine.slic(lab, c["S"], 0.6, it)
        _, osp, olb = orc.slic(b["stack"][0], c["S"], 0.6, it)
        assert_bits(as_u32(lb)[0], olb, f"labels it{it}")
        assert_bits(sp.cpu().numpy()[0][..., :7], osp[..., :7], f"spixl it{it}")


def _chain(engine, c, b):
    lab, _ = engine.cvt(dev(b["stack"]))
    sp, lb = engine.slic(lab, c["S"], 0.6, 5)
    rep = engine.boundary(sp, lb, c["S"])
    return lab, sp, lb, rep


@pytest.mark.parametrize("name", list(CASES))
def test_boundary_and_sweep(engine, name):
    c = CASES[name]
    b = build(c)
    lab, sp, lb, rep = _chain(engine, c, b)
    lab_h, sp_h, lb_h = lab.cpu().numpy(), sp.cpu().numpy(), as_u32(lb)
    orep = orc.boundary(sp_h, lb_h, c["S"])
    assert_bits(rep.cpu().numpy(), orep, "rep")
    cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], b["sn"])
    engine.sweep_spixl(lab, sp, rep, cam, c["S"])
    osp = orc.sweep(lab_h, sp_h, orep, b["levels"], b["vs"], b["sn"], c["aw"], c["bl"], c["S"])
    assert_bits(sp.cpu().numpy()[..., 7], osp[..., 7], "s7")


@pytest.mark.parametrize("dmax", [31, 32, 47, 100, 200])
def test_sweep_level_counts(engine, dmax):
    """k_sweep_spixl's lane layouts by level count: two superpixels per wave
    (D <= 32), one wave (D <= 64), two or four waves per superpixel."""
    c = dict(CASES["c3x1_s16"], dmin=0, dmax=dmax, seed=41)
    b = build(c)
    lab, sp, lb, rep = _chain(engine, c, b)
    lab_h, sp_h, lb_h = lab.cpu().numpy(), sp.cpu().numpy(), as_u32(lb)
    orep = orc.boundary(sp_h, lb_h, c["S"])
    cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], b["sn"])
    engine.sweep_spixl(lab, sp, rep, cam, c["S"])
    osp = orc.sweep(lab_h, sp_h, orep, b["levels"], b["vs"], b["sn"], c["aw"], c["bl"], c["S"])
    assert_bits(sp.cpu().numpy()[..., 7], osp[..., 7], f"s7 D={dmax + 1}")


@pytest.mark.parametrize("name", list(PIXEL_CASES))
def test_grid_and_pixel_sad(engine, name):
    c = PIXEL_CASES[name]
    b = build(c)
    lab, _ = engine.cvt(dev(b["stack"]))
    sp, lb = engine.grid(lab, 1)
    for v in range(b["V"]):
        _, osp, olb = orc.grid(b["stack"][v], 1)
        assert_bits(as_u32(lb)[v], olb, "grid labels")
        assert_bits(sp.cpu().numpy()[v][..., :7], osp[..., :7], "grid spixl")
    cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], b["sn"])
    disp = engine.sweep_pixel_sad(lab, cam)
    want = orc.sweep_pixel_sad(lab.cpu().numpy(), b["levels"], b["vs"], b["sn"], c["aw"], c["bl"])
    assert_bits(disp.cpu().numpy(), want, "per-pixel SAD disparity")
    # and the generic superpixel sweep on the S=1 grid gives the same map
    rep = engine.boundary(sp, lb, 1)
    engine.sweep_spixl(lab, sp, rep, cam, 1)
    assert_bits(sp.cpu().numpy()[..., 7], want, "grid sweep == per-pixel sweep")


def test_cvt_every_rgb_colour(engine):
    """k_cvt on all 2^24 8-bit colours (one 4096x4096 RGBx image) against the
    oracle: the cube-root fast path (slic.hip powr_third) must round exactly as
    the definition mvs_powrf does, and the 8-bit NCC intensity follows L."""
    v = np.arange(1 << 24, dtype=np.uint32)
    rgbx = np.zeros((1, 4096, 4096, 4), np.uint8)
    flat = rgbx[0].reshape(-1, 4)
    flat[:, 0], flat[:, 1], flat[:, 2] = v & 255, (v >> 8) & 255, v >> 16
    lab, l8 = engine.cvt(dev(rgbx))
    want = orc.cvt(rgbx)
    assert_bits(lab.cpu().numpy(), want, "Lab of every colour")
    assert_bits(l8.cpu().numpy(), orc.l8(want), "l8 of every colour")


@pytest.mark.parametrize("K", [5, 7])
@pytest.mark.parametrize("name", ["c2x1_pix", "c2x2_pix", "c3x1_pix_odd", "c5x1_ncc", "c4x1_ncc_d40", "c3x1_inc3"])
def test_ncc_volume_and_wta(engine, name, K):
    if name == "c5x1_ncc":
        c = dict(aw=5, ah=1, W=150, H=70, dmin=0, dmax=20, bl=1.0, nh=4, nv=0, seed=23)
    elif name == "c4x1_ncc_d40":  # odd width, 40 levels, |dx| up to 3 (partial residue tiles)
        c = dict(aw=4, ah=1, W=131, H=37, dmin=3, dmax=42, bl=1.0, nh=3, nv=0, seed=29)
    elif name == "c3x1_inc3":  # level step 3: shifts 3|dx| per level
        c = dict(aw=3, ah=1, W=97, H=41, dmin=1, dmax=31, inc=3, bl=1.0, nh=2, nv=0, seed=31)
    else:
        c = PIXEL_CASES[name]
    b = build(c)
    lab, l8 = engine.cvt(dev(b["stack"]))
    box = engine.box_stats(l8, K)
    cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], b["sn"])
    l8h = l8.cpu().numpy()
    assert_bits(l8h, orc.l8(lab.cpu().numpy()), "l8")
    lv = engine.levels_dev(cam)
    for z in range(b["V"]):
        vol = engine.ncc_volume(l8, box, cam, z, K)
        want = orc.ncc_volume(l8h, b["levels"], b["vs"], b["sn"], c["aw"], c["bl"], K, z)
        assert_bits(vol.cpu().numpy(), want, f"ncc volume z{z}")
        disp, conf = engine.wta(vol, lv)
        od, oc = orc.wta(want, b["levels"])
        assert_bits(disp.cpu().numpy(), od, "wta disp")
        assert_bits(conf.cpu().numpy(), oc, "wta conf")
        fd, fc = engine.ncc_wta(l8, box, cam, z, K)  # fused: no volume
        assert_bits(fd.cpu().numpy(), od, "fused wta disp")
        assert_bits(fc.cpu().numpy(), oc, "fused wta conf")


@pytest.mark.parametrize("name,dmax,flat", [("d1", 0, False), ("d2", 1, False), ("d3", 2, True), ("d5", 4, False),
                                            ("d9_flat", 8, True), ("d33_flat", 32, True), ("d70", 69, False)])
def test_ncc_wta_fused_edges(engine, name, dmax, flat):
    """Fused sweep+WTA vs the oracle's volume + WTA at level counts below /
    around the NW=8 waves x DPW=4 chunk, and with textureless (constant)
    patches, whose cost ties (cost 1 at every level) exercise the first-argmin
    tie rule across waves.  View 0 of a 3x1 array with no neighbours listed
    exercises the every-window-invalid path."""
    c = dict(aw=3, ah=1, W=133, H=29, dmin=0, dmax=dmax, bl=1.0, nh=2, nv=0, seed=37)
    b = build(c)
    stack = b["stack"].copy()
    if flat:
        stack[:, 5:20, 10:70, :3] = 128
        stack[1, :, 90:120, :3] = 40
    sn = b["sn"].copy()
    sn[0] = 0
    lab, l8 = engine.cvt(dev(stack))
    cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], sn)
    l8h = l8.cpu().numpy()
    for K in (5, 7):
        box = engine.box_stats(l8, K)
        for z in range(b["V"]):
            want = orc.ncc_volume(l8h, b["levels"], b["vs"], sn, c["aw"], c["bl"], K, z)
            od, oc = orc.wta(want, b["levels"])
            fd, fc = engine.ncc_wta(l8, box, cam, z, K)
            assert_bits(fd.cpu().numpy(), od, f"fused disp K{K} z{z}")
            assert_bits(fc.cpu().numpy(), oc, f"fused conf K{K} z{z}")
            fd2, _ = engine.ncc_wta(l8, box, cam, z, K, want_conf=False)
            assert_bits(fd2.cpu().numpy(), od, f"fused disp (no conf) K{K} z{z}")


@pytest.mark.parametrize("name,ks,kst", [("c3x3_s8", 26, 13), ("c3x1_s16", 52, 13), ("c5x1_s32", 1080, 13),
                                         ("c3x1_s8", 1080, 13), ("c5x3_s16", 1080, 13),
                                         ("c3x1_s8", 1080, 16)])  # kernel_step 16: > 64 smoothness terms
def test_refinement(engine, name, ks, kst):
    c = CASES[name]
    b = build(c)
    lab, sp, lb, rep = _chain(engine, c, b)
    cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], b["sn"])
    engine.sweep_spixl(lab, sp, rep, cam, c["S"])
    sp_h, lb_h, rep_h = sp.cpu().numpy(), as_u32(lb), rep.cpu().numpy()
    want = orc.refine(sp_h, lb_h, rep_h, b["vs"], b["sn"], c["aw"], c["bl"], c["S"], 2.0, 6.0, 1.0, kst, ks, 5, True)
    got = engine.refine(sp, lb, rep, cam, c["S"], 2.0, 6.0, 1.0, kst, ks, 5, True)
    assert_bits(got["flat"].cpu().numpy(), want["flat"], "flatness")
    assert_bits(got["state_compat"].cpu().numpy(), want["states"][3], "state after iteration 3 (fusion input)")
    assert_bits(got["disp"].cpu().numpy(), want["disp"], "fused disparity")
    # per-stage: init state and each propagate iteration
    rp = params.refine_params(params.Settings(spixl_size=c["S"], kernel_size=ks, kernel_step=kst))
    flat = engine.flatness(sp, rp["flat_gamma"])
    st = engine.init_state(sp, lb, rep, flat, cam, c["S"], rp["init_gamma"], rp["init_alpha"], rp["kernel_steps"],
                           rp["kss"], rp["fuse"])
    assert_bits(st.cpu().numpy(), want["state0"], "init state")
    cur = st
    for it in range(5):
        nks, kss = params.prop_schedule(it, rp["kernel_steps"], rp["kss"])
        nxt = torch.empty_like(cur)
        engine.propagate(sp, lb, rep, flat, cam, c["S"], it, rp["prop_alpha"], rp["prop_gamma"], rp["fuse"], nks, kss,
                         cur, nxt)
        assert_bits(nxt.cpu().numpy(), want["states"][it], f"propagate iteration {it}")
        cur = nxt


def _refine_stages(engine, sp, lb, rep, cam, S, ks=1080, kst=13):
    """init state, the 5 propagate iterations and the fused map, with the
    refinement's parameters: the entry points chosen by the labels' dtype."""
    V = lb.shape[0]
    rp = params.refine_params(params.Settings(spixl_size=S, kernel_size=ks, kernel_step=kst))
    flat = engine.flatness(sp, rp["flat_gamma"])
    cur = engine.init_state_range(sp, lb, rep, flat, cam, S, rp["init_gamma"], rp["init_alpha"], rp["kernel_steps"],
                                  rp["kss"], rp["fuse"], 0, V)
    out = [cur.clone()]
    for it in range(5):
        nks, kss = params.prop_schedule(it, rp["kernel_steps"], rp["kss"])
        nxt = torch.empty_like(cur)
        engine.propagate(sp, lb, rep, flat, cam, S, it, rp["prop_alpha"], rp["prop_gamma"], rp["fuse"], nks, kss,
                         cur, nxt)
        out.append(nxt)
        cur = nxt
    out.append(engine.spixl_to_image(sp, lb, cur, S))
    return [t.cpu().numpy() for t in out]


@pytest.mark.parametrize("name", ["c3x3_s8", "c5x1_s32"])
def test_refinement_labels16(engine, name):
    """The 16-bit label entry points (the sharded pipeline's narrowed labels,
    ABI 0.5) against the oracle, stage by stage."""
    c = CASES[name]
    b = build(c)
    lab, sp, lb, rep = _chain(engine, c, b)
    cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], b["sn"])
    engine.sweep_spixl(lab, sp, rep, cam, c["S"])
    want = orc.refine(sp.cpu().numpy(), as_u32(lb), rep.cpu().numpy(), b["vs"], b["sn"], c["aw"], c["bl"], c["S"],
                      2.0, 6.0, 1.0, 13, 1080, 5, True)
    got = _refine_stages(engine, sp, lb.to(torch.int16).view(torch.uint16), rep, cam, c["S"])
    assert_bits(got[0], want["state0"], "init state (16-bit labels)")
    for it in range(5):
        assert_bits(got[1 + it], want["states"][it], f"propagate iteration {it} (16-bit labels)")


@pytest.mark.parametrize("W", [400, 398])  # 398: the one-pixel fusion kernel (W % 4 != 0)
def test_labels16_above_32767(engine, W):
    """Labels with the top bit of 16 set (S = 2: 40,000 superpixels per view)
    read unsigned: every stage equal to the uint32 entry points bit for bit."""
    S = 2
    stack, _ = synth.make_stack(W, 400, 3, 1, 0, 15, 1.0, 5)
    vs, sn = params.flatten_subsets(params.neighbour_lists(3, 1, 1, 0))
    cam = CameraArray(3, 1.0, params.disparity_levels(0, 15, 1), vs, sn)
    lab, _ = engine.cvt(dev(stack))
    sp, lb = engine.grid(lab, S)
    rep = engine.boundary(sp, lb, S)
    engine.sweep_spixl(lab, sp, rep, cam, S)
    assert int(lb.max()) >= 1 << 15
    want = _refine_stages(engine, sp, lb, rep, cam, S)
    got = _refine_stages(engine, sp, lb.to(torch.int16).view(torch.uint16), rep, cam, S)
    for k, (g, w) in enumerate(zip(got, want)):
        assert_bits(g, w, f"stage {k} (16-bit vs 32-bit labels)")
    with pytest.raises(Exception, match="bad arguments"):  # 16-bit maps need mw * mh <= 65536
        sp1, lb1 = engine.grid(lab, 1)
        engine.spixl_to_image(sp1, lb1.to(torch.int16), torch.zeros(3, 400, W, 6, device="cuda"), 1)


@pytest.mark.parametrize("name", ["c3x3_s8", "c3x1_s16"])
def test_filter(engine, name):
    c = CASES[name]
    b = build(c)
    rng = np.random.default_rng(5)
    V = b["V"]
    disp = rng.integers(c["dmin"], c["dmax"] + 1, size=(V, c["H"], c["W"])).astype(np.float32)
    disp[rng.random(disp.shape) < 0.05] = 0.0
    disp += rng.choice(np.float32([0.0, 0.25, 0.5]), size=disp.shape)
    proj, out = engine.filter(dev(disp), c["aw"], c["bl"], 1.0)
    oproj, oout = orc.filt(disp, c["aw"], c["bl"], 1.0)
    assert_bits(proj.cpu().numpy(), oproj, "filter projection")
    assert_bits(out.cpu().numpy(), oout, "filter output")


@pytest.mark.parametrize("aw,ah", [(8, 4), (9, 5), (10, 7)])
def test_filter_many_views(engine, aw, ah):
    # V = 32 / 45 / 70: the candidate-selection kernel at MAXV 32 and 64, and
    # the direct kernel past 64 views; smooth disparities with ties, zeros and
    # out-of-image projections
    V, H, W = aw * ah, 24, 40
    rng = np.random.default_rng(aw * 10 + ah)
    base = rng.integers(2, 9, size=(V, 1, 1)).astype(np.float32)
    disp = base + rng.choice(np.float32([0.0, 0.5, 1.0, 3.0]), size=(V, H, W))
    disp[rng.random(disp.shape) < 0.1] = 0.0
    proj, out = engine.filter(dev(disp), aw, 1.0, 1.0)
    oproj, oout = orc.filt(disp, aw, 1.0, 1.0)
    assert_bits(proj.cpu().numpy(), oproj, "filter projection")
    assert_bits(out.cpu().numpy(), oout, "filter output")


@pytest.mark.parametrize("kern,fb,ns,bound", [("q", 2, 2, 1), ("q", 4, 2, 1), ("q", 2, 1, 1), ("q", 4, 1, 1),
                                               ("q", 2, 2, 0), ("px", 4, 0, 1), ("px", 2, 0, 1)])
@pytest.mark.parametrize("aw,ah", [(8, 4), (6, 5), (5, 5)])
def test_filter_variants(engine, monkeypatch, aw, ah, kern, fb, ns, bound):
    # every removal kernel for 16 < V <= 32, forced per call (MVS_FILTER_KERNEL /
    # _FB / _NS / _BOUND are read at each launch): the per-lane queue walk (1
    # or 2 candidate slots, with and without the in-image bounds), with
    # row-shared (aw % FB == 0) and per-view offsets, and the per-pixel form.
    # Near-equal candidates in long runs reach the queue kernel's full-count
    # fallback of the first stability term.
    V, H, W = aw * ah, 20, 72
    rng = np.random.default_rng(aw * 100 + ah * 7 + fb)
    base = rng.integers(2, 12, size=(V, 1, 1)).astype(np.float32)
    disp = base + rng.choice(np.float32([0.0, 0.25, 0.5, 1.0, 1.5, 6.0]), size=(V, H, W))
    disp[:, :4] = 5.0 + rng.choice(np.float32([0.0, 0.5]), size=(V, 4, W))  # long runs within fuse
    disp[rng.random(disp.shape) < 0.1] = 0.0
    monkeypatch.setenv("MVS_FILTER_KERNEL", kern)
    monkeypatch.setenv("MVS_FILTER_FB", str(fb))
    monkeypatch.setenv("MVS_FILTER_NS", str(ns))
    monkeypatch.setenv("MVS_FILTER_BOUND", str(bound))
    proj, out = engine.filter(dev(disp), aw, 1.0359, 1.0)
    oproj, oout = orc.filt(disp, aw, 1.0359, 1.0)
    assert_bits(proj.cpu().numpy(), oproj, "filter projection")
    assert_bits(out.cpu().numpy(), oout, f"filter output ({kern}, FB {fb})")


@pytest.mark.parametrize("bound", [1, 0])
def test_filter_signed_far_disparities(engine, monkeypatch, bound):
    # negative and far disparities (|d| up to 300 on a 72 x 20 image): the queue
    # walk's in-image intervals with reversed ends (d < 0) and ends clamped to
    # int8, candidates with no in-image view at all, every view out of image
    V, aw, H, W = 32, 8, 20, 72
    rng = np.random.default_rng(4242 + bound)
    disp = rng.choice(np.float32([-300.0, -40.0, -7.5, -2.0, -0.5, 0.5, 2.0, 7.5, 40.0, 300.0]), size=(V, H, W))
    disp += rng.choice(np.float32([0.0, 0.25, 0.5]), size=(V, H, W))
    disp[rng.random(disp.shape) < 0.15] = 0.0
    monkeypatch.setenv("MVS_FILTER_KERNEL", "q")
    monkeypatch.setenv("MVS_FILTER_BOUND", str(bound))
    proj, out = engine.filter(dev(disp), aw, 1.0359, 1.0)
    oproj, oout = orc.filt(disp, aw, 1.0359, 1.0)
    assert_bits(proj.cpu().numpy(), oproj, "filter projection")
    assert_bits(out.cpu().numpy(), oout, f"filter output (signed far disparities, bound {bound})")


@pytest.mark.parametrize("fb,ns", [(2, 2), (4, 1)])
def test_filter_ragged_grid(engine, monkeypatch, fb, ns):
    # V = 27 views on rows of aw = 6 (the last camera row holds 3): the queue
    # walk's row-shared (FB 2) and per-view (FB 4) offsets over j < V, without
    # the in-image bounds (they assume a complete aw x (V / aw) grid)
    V, aw, H, W = 27, 6, 20, 72
    rng = np.random.default_rng(27 + fb)
    base = rng.integers(2, 12, size=(V, 1, 1)).astype(np.float32)
    disp = base + rng.choice(np.float32([0.0, 0.25, 0.5, 1.0, 1.5, 6.0]), size=(V, H, W))
    disp[rng.random(disp.shape) < 0.1] = 0.0
    monkeypatch.setenv("MVS_FILTER_KERNEL", "q")
    monkeypatch.setenv("MVS_FILTER_FB", str(fb))
    monkeypatch.setenv("MVS_FILTER_NS", str(ns))
    proj, out = engine.filter(dev(disp), aw, 1.0359, 1.0)
    oproj, oout = orc.filt(disp, aw, 1.0359, 1.0)
    assert_bits(proj.cpu().numpy(), oproj, "filter projection")
    assert_bits(out.cpu().numpy(), oout, f"filter output (ragged grid, FB {fb})")


@pytest.mark.parametrize("kern,aw,ah", [("q", 3, 2), ("q", 4, 3), ("q", 8, 4), ("q", 9, 5), ("q", 10, 7),
                                         ("px", 8, 4)])
def test_filter_row_bands(engine, monkeypatch, aw, ah, kern):
    # mvs_proj_inv_rows_d / mvs_remove_inconsistency_rows_d (the sharded
    # pipeline's banded proj all-gather): uneven row bands, every band written
    # into shared proj / out buffers, tile the full-range result for every
    # removal kernel (V = 6, 12, 32, 45, 70; the 16 < V <= 32 kernels forced
    # per call), the projection into the full stack and into band buffers
    V, H, W = aw * ah, 23, 70  # the "px" removal variant is forced only at 16 < V <= 32 (8 x 4)
    rng = np.random.default_rng(aw * 13 + ah)
    base = rng.integers(2, 9, size=(V, 1, 1)).astype(np.float32)
    disp = base + rng.choice(np.float32([0.0, 0.5, 1.0, 3.0]), size=(V, H, W))
    disp[rng.random(disp.shape) < 0.1] = 0.0
    d = dev(disp)
    monkeypatch.setenv("MVS_FILTER_KERNEL", kern)
    oproj, oout = orc.filt(disp, aw, 1.0359, 1.0)
    bands = [(0, 5), (5, 6), (6, 17), (17, 17), (17, 23)]
    proj = torch.full((V, H, W), float("nan"), device=d.device)
    for ya, yb in bands:
        engine.proj_inv(d, aw, 1.0359, 0, V, proj=proj, rows=(ya, yb))
    assert_bits(proj.cpu().numpy(), oproj, "banded projection")
    for z0, z1 in ((0, V // 3), (V // 3, V)):  # straight into band buffers, [V, yb - ya, W]
        for ya, yb in bands:
            buf = torch.full((V, yb - ya, W), float("nan"), device=d.device)
            engine.proj_inv(d, aw, 1.0359, z0, z1, proj=buf, rows=(ya, yb), band=True)
            assert_bits(buf[z0:z1].cpu().numpy(), oproj[z0:z1, ya:yb], "band-buffer projection")
    for band in (False, True):  # proj rows within the full stack / the band alone, [V, yb - ya, W]
        out = torch.full((V, H, W), -1.0, device=d.device)
        for z0, z1 in ((0, V // 3), (V // 3, V)):
            for ya, yb in bands:
                pj = proj[:, ya:yb].contiguous() if band else proj
                engine.remove_inconsistency(d, pj, aw, 1.0359, 1.0, z0, z1, out=out, rows=(ya, yb), band=band)
        assert_bits(out.cpu().numpy(), oout, f"banded removal ({kern}, band buffer {band})")


def test_determinism(engine):
    c = CASES["c5x1_s32"]
    b = build(c)
    outs = []
    for _ in range(2):
        lab, sp, lb, rep = _chain(engine, c, b)
        outs.append((sp.cpu().numpy().copy(), as_u32(lb).copy()))
    assert_bits(outs[0][0], outs[1][0], "spixl rerun")
    assert_bits(outs[0][1], outs[1][1], "labels rerun")


def test_host_api_matches_device_api(engine):
    """mvs_do_super_pixel_seg (host pointers) == device path."""
    import ctypes as C
    from cl_multiview_stereo_amd import _lib
    c = CASES["c3x1_s16"]
    b = build(c)
    img = np.ascontiguousarray(b["stack"][0])
    H, W = img.shape[:2]
    mw, mh = params.map_size(W, H, c["S"])
    lab = np.zeros((H, W, 4), np.float32)
    sp = np.zeros((mh, mw, 8), np.float32)
    lb = np.zeros((H, W), np.uint32)
    p = _lib.SlicParams(c["S"], 0.6, 5, 0, 0)
    _lib.check(engine.L.mvs_do_super_pixel_seg(engine.ctx, img.ctypes.data_as(C.c_void_p), W, H, C.byref(p),
                                               lab.ctypes.data_as(C.c_void_p), sp.ctypes.data_as(C.c_void_p),
                                               lb.ctypes.data_as(C.c_void_p)), "mvs_do_super_pixel_seg")
    olab, osp, olb = orc.slic(img, c["S"])
    assert_bits(lb, olb, "host-API labels")
    assert_bits(sp[..., :7], osp[..., :7], "host-API spixl")


def test_bad_arguments_fail_loudly(engine):
    from cl_multiview_stereo_amd import _lib
    lab = torch.zeros((1, 16, 16, 4), device="cuda")
    with pytest.raises(_lib.MvsError):
        engine.slic(lab, 4)  # S < 6: the reference update divides by 3S/16 == 0


def test_full_size_slic_properties(engine):
    """1080p, S=32 (BASELINE config 2): labels in range, every label is one of
    the pixel's candidate centres, and a rerun is bit-identical."""
    stack, _ = synth.make_stack(1920, 1080, 5, 1, 0, 127, 1.0, 0x5EED + 2)
    lab, _ = engine.cvt(dev(stack))
    sp, lb = engine.slic(lab, 32)
    sp2, lb2 = engine.slic(lab, 32)
    assert torch.equal(lb, lb2) and torch.equal(sp, sp2)
    lbh = as_u32(lb)
    mw, mh = params.map_size(1920, 1080, 32)
    assert lbh.max() < mw * mh
    ys, xs = np.mgrid[0:1080, 0:1920]
    lx, ly = lbh[0] % mw, lbh[0] // mw
    assert np.all(np.abs(lx - xs // 32) <= 1) and np.all(np.abs(ly - ys // 32) <= 1)
    # one view against the oracle at full size
    olab, osp, olb = orc.slic(stack[0], 32)
    assert_bits(lbh[0], olb, "1080p labels")


@pytest.mark.parametrize("S", [32, 48, 64])
@pytest.mark.parametrize("tiles9", ["0", "1"])
def test_slic_tile_kernels(engine, monkeypatch, S, tiles9):
    """The tile-fused assignment kernels against the oracle, labels and centres
    bit for bit, on an image whose size is a multiple of neither 16 nor S:
    k_assign_tiles4<S / 16> (S = 32, 64: the tile's four candidate cells,
    branch-free distances, packed trees of the joined cells only) and the
    9-cell k_assign_tiles (S = 48, whose tiles can straddle a candidate
    boundary, or any S with MVS_SLIC_TILES9=1)."""
    monkeypatch.setenv("MVS_SLIC_TILES9", tiles9)
    W, H = 330, 250
    stack, _ = synth.make_stack(W, H, 2, 1, 0, 15, 1.0, 31 + S)
    lab, _ = engine.cvt(dev(stack))
    sp, lb = engine.slic(lab, S, 0.6, 5)
    sp, lb = sp.cpu().numpy(), as_u32(lb)
    for v in range(2):
        _, osp, olb = orc.slic(stack[v], S, 0.6, 5)
        assert_bits(lb[v], olb, f"labels S={S} v{v}")
        assert_bits(sp[v][..., :7], osp[..., :7], f"spixl S={S} v{v}")


@pytest.mark.parametrize("kind", ["flat", "ramp", "checker"])
def test_slic_ties(engine, kind):
    """Images built so that many pixels sit at (near-)equal distance from two
    candidate centres: the assignment's strict-< first-wins tie rule and the
    lazily evaluated square roots must still give the oracle's labels."""
    H, W, S = 96, 128, 16
    y, x = np.mgrid[0:H, 0:W]
    if kind == "flat":
        img = np.full((H, W, 3), 120, np.uint8)
    elif kind == "ramp":
        img = np.stack([(x * 2) % 256, (y * 2) % 256, ((x + y) // 2) % 256], -1).astype(np.uint8)
    else:
        img = np.where(((x // 8 + y // 8) % 2)[..., None] == 0, 40, 200).astype(np.uint8).repeat(3, -1)
    rgbx = np.concatenate([img, np.zeros((H, W, 1), np.uint8)], -1)[None]
    lab, _ = engine.cvt(dev(rgbx))
    for S_ in (S, 32, 8, 64):
        sp, lb = engine.slic(lab, S_)
        _, osp, olb = orc.slic(rgbx[0], S_)
        assert_bits(as_u32(lb)[0], olb, f"{kind} labels S={S_}")
        assert_bits(sp.cpu().numpy()[0][..., :7], osp[..., :7], f"{kind} spixl S={S_}")


@pytest.mark.parametrize("name", ["c3x1_s16", "c3x3_s8"])
def test_concurrent_pipeline_matches_serial(engine, name):
    """Pipeline(concurrent=True) runs the superpixel chain on a second stream
    and context, fused=True folds the WTA into the sweep: every output equals
    the one-stream two-pass pipeline's bit for bit."""
    from cl_multiview_stereo_amd.pipeline import Pipeline
    c = CASES[name]
    b = build(c)
    st = params.Settings(spixl_size=c["S"], array_width=c["aw"], array_height=c["ah"], min_disp=c["dmin"],
                         max_disp=c["dmax"], inc=1, neib_hor=c["nh"], neib_ver=c["nv"], bl_ratio=c["bl"], window=5,
                         cost="ncc")
    rgbx = dev(b["stack"])
    outs = []
    for conc, fused in ((False, False), (True, False), (False, True), (True, True)):
        p = Pipeline(engine, st, c["W"], c["H"], concurrent=conc, fused=fused)
        o = p.exe_pipeline(rgbx)
        o = p.exe_pipeline(rgbx)  # twice: the second run reuses cached allocator blocks across streams
        torch.cuda.synchronize()
        outs.append(o)
    for o in outs[1:]:
        for f in ("spixl", "labels", "rep", "disp", "conf"):
            assert_bits(getattr(o, f).cpu().numpy(), getattr(outs[0], f).cpu().numpy(), f)
