"""Committed golden fixtures (tests/golden/*.npz, made by gen_fixtures.py):
the CPU oracle must still reproduce them (CPU suite) and the HIP path must
reproduce them bit-for-bit through the C-ABI (GPU suite)."""
from __future__ import annotations

import hashlib
import os

import numpy as np
import pytest

from oracle import oracle as orc

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(GOLD, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def same(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if a.dtype == np.float32:
        a, b = a.view(np.uint32), np.asarray(b, np.float32).view(np.uint32)
    return a.shape == b.shape and np.array_equal(a, b)


# ------------------------------------------------------------------ CPU ---
def test_oracle_reproduces_spixl_fixture():
    g = load("spixl_c3x1_s8.npz")
    aw, ah, W, H, S, ks = (int(v) for v in g["meta"])
    bl = float(g["bl"])
    outs = [orc.slic(g["rgbx"][v], S) for v in range(len(g["rgbx"]))]
    lab = np.stack([o[0] for o in outs])
    sp = np.stack([o[1] for o in outs])
    lb = np.stack([o[2] for o in outs])
    assert sha(lab) == str(g["lab_sha"])
    assert same(lb, g["labels"])
    rep = orc.boundary(sp, lb, S)
    assert same(rep, g["rep"])
    sp = orc.sweep(lab, sp, rep, g["levels"], g["view_subset"], g["subset_num"], aw, bl, S)
    assert same(sp, g["spixl"])
    ref = orc.refine(sp, lb, rep, g["view_subset"], g["subset_num"], aw, bl, S, kernel_size=ks)
    for k in ("flat", "state0", "states", "disp"):
        assert same(ref[k], g[k]), k
    proj, filt = orc.filt(ref["disp"], aw, bl, 1.0)
    assert same(proj, g["proj"]) and same(filt, g["filt"])


def test_oracle_reproduces_pixel_fixture():
    g = load("pixel_c2x2_ncc5.npz")
    aw, ah, W, H, K = (int(v) for v in g["meta"])
    bl = float(g["bl"])
    lab = orc.cvt(g["rgbx"])
    q = orc.l8(lab)
    assert same(q, g["l8"])
    for z in range(len(q)):
        vol = orc.ncc_volume(q, g["levels"], g["view_subset"], g["subset_num"], aw, bl, K, z)
        assert sha(vol) == str(g["vol_sha"][z])
        if z == 0:
            assert same(vol, g["vol0"])
        d, c = orc.wta(vol, g["levels"])
        assert same(d, g["disp"][z]) and same(c, g["conf"][z])
    assert same(orc.sweep_pixel_sad(lab, g["levels"], g["view_subset"], g["subset_num"], aw, bl), g["sad"])


def test_fixture_files_are_plain_arrays():
    for f in os.listdir(GOLD):
        if f.endswith(".npz"):
            g = load(f)  # allow_pickle=False: no object arrays
            assert all(v.dtype != object for v in g.values())


# ------------------------------------------------------------------ GPU ---
@pytest.mark.gpu
def test_gpu_reproduces_spixl_fixture(engine):
    import torch
    from cl_multiview_stereo_amd.engine import CameraArray
    g = load("spixl_c3x1_s8.npz")
    aw, ah, W, H, S, ks = (int(v) for v in g["meta"])
    bl = float(g["bl"])
    lab, _ = engine.cvt(torch.from_numpy(g["rgbx"]).cuda())
    assert sha(lab.cpu().numpy()) == str(g["lab_sha"])
    sp, lb = engine.slic(lab, S)
    assert same(lb.cpu().numpy().view(np.uint32), g["labels"])
    rep = engine.boundary(sp, lb, S)
    assert same(rep.cpu().numpy(), g["rep"])
    cam = CameraArray(aw, bl, g["levels"], g["view_subset"], g["subset_num"])
    engine.sweep_spixl(lab, sp, rep, cam, S)
    assert same(sp.cpu().numpy()[..., 7], g["spixl"][..., 7])
    out = engine.refine(sp, lb, rep, cam, S, 2.0, 6.0, 1.0, 13, ks, 5, True)
    assert same(out["flat"].cpu().numpy(), g["flat"])
    assert same(out["state_compat"].cpu().numpy(), g["states"][3])
    assert same(out["disp"].cpu().numpy(), g["disp"])
    proj, filt = engine.filter(out["disp"], aw, bl, 1.0)
    assert same(proj.cpu().numpy(), g["proj"]) and same(filt.cpu().numpy(), g["filt"])


@pytest.mark.gpu
def test_gpu_reproduces_pixel_fixture(engine):
    import torch
    from cl_multiview_stereo_amd.engine import CameraArray
    g = load("pixel_c2x2_ncc5.npz")
    aw, ah, W, H, K = (int(v) for v in g["meta"])
    bl = float(g["bl"])
    lab, l8 = engine.cvt(torch.from_numpy(g["rgbx"]).cuda())
    assert same(l8.cpu().numpy(), g["l8"])
    box = engine.box_stats(l8, K)
    cam = CameraArray(aw, bl, g["levels"], g["view_subset"], g["subset_num"])
    lv = engine.levels_dev(cam)
    for z in range(len(g["rgbx"])):
        vol = engine.ncc_volume(l8, box, cam, z, K)
        assert sha(vol.cpu().numpy()) == str(g["vol_sha"][z])
        d, c = engine.wta(vol, lv)
        assert same(d.cpu().numpy(), g["disp"][z]) and same(c.cpu().numpy(), g["conf"][z])
    disp = engine.sweep_pixel_sad(lab, cam)
    assert same(disp.cpu().numpy(), g["sad"])
