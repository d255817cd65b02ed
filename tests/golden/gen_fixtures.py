"""Generate the committed golden fixtures under tests/golden/.

Test infrastructure.  The reference has no tests, fixtures or golden vectors
of its own, and running the reference itself is not
available to this build, so these vectors come from the
CPU oracle (oracle/mvs_oracle.c, cross-checked bit-for-bit by the independent
numpy restatement in tests/np_ref.py).  They freeze the definition: a later
change to either the oracle or the HIP kernels that moves any output bit
fails tests/test_golden.py.

    python tests/golden/gen_fixtures.py      # rewrites tests/golden/*.npz
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from cl_multiview_stereo_amd import params, synth  # noqa: E402
from oracle import oracle as orc  # noqa: E402

# superpixel path: SLIC -> boundary -> sweep -> refinement -> filter
SPIXL = dict(aw=3, ah=1, W=100, H=70, S=8, dmin=0, dmax=15, bl=1.0, nh=1, nv=1, seed=11, ks=1080)
# per-pixel path: l8 -> NCC 5x5 volume -> WTA, and the S=1 SAD parity sweep
PIXEL = dict(aw=2, ah=2, W=48, H=40, dmin=0, dmax=9, bl=1.0359, nh=1, nv=1, seed=16, K=5)


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def spixl_fixture():
    c = SPIXL
    stack, _ = synth.make_stack(c["W"], c["H"], c["aw"], c["ah"], c["dmin"], c["dmax"], c["bl"], c["seed"])
    levels = params.disparity_levels(c["dmin"], c["dmax"], 1)
    vs, sn = params.flatten_subsets(params.neighbour_lists(c["aw"], c["ah"], c["nh"], c["nv"]))
    outs = [orc.slic(stack[v], c["S"]) for v in range(len(stack))]
    lab = np.stack([o[0] for o in outs])
    sp = np.stack([o[1] for o in outs])
    lb = np.stack([o[2] for o in outs])
    rep = orc.boundary(sp, lb, c["S"])
    sp = orc.sweep(lab, sp, rep, levels, vs, sn, c["aw"], c["bl"], c["S"])
    ref = orc.refine(sp, lb, rep, vs, sn, c["aw"], c["bl"], c["S"], kernel_size=c["ks"])
    proj, filt = orc.filt(ref["disp"], c["aw"], c["bl"], 1.0)
    np.savez_compressed(
        os.path.join(HERE, "spixl_c3x1_s8.npz"),
        rgbx=stack, levels=levels, view_subset=vs, subset_num=sn,
        meta=np.array([c["aw"], c["ah"], c["W"], c["H"], c["S"], c["ks"]], np.int32), bl=np.float32(c["bl"]),
        lab_sha=np.array(sha(lab)), labels=lb, spixl=sp, rep=rep, flat=ref["flat"], state0=ref["state0"],
        states=ref["states"], disp=ref["disp"], proj=proj, filt=filt)


def pixel_fixture():
    c = PIXEL
    stack, _ = synth.make_stack(c["W"], c["H"], c["aw"], c["ah"], c["dmin"], c["dmax"], c["bl"], c["seed"])
    levels = params.disparity_levels(c["dmin"], c["dmax"], 1)
    vs, sn = params.flatten_subsets(params.neighbour_lists(c["aw"], c["ah"], c["nh"], c["nv"]))
    lab = orc.cvt(stack)
    q = orc.l8(lab)
    V = len(stack)
    vols = [orc.ncc_volume(q, levels, vs, sn, c["aw"], c["bl"], c["K"], z) for z in range(V)]
    wt = [orc.wta(v, levels) for v in vols]
    sad = orc.sweep_pixel_sad(lab, levels, vs, sn, c["aw"], c["bl"])
    np.savez_compressed(
        os.path.join(HERE, "pixel_c2x2_ncc5.npz"),
        rgbx=stack, levels=levels, view_subset=vs, subset_num=sn,
        meta=np.array([c["aw"], c["ah"], c["W"], c["H"], c["K"]], np.int32), bl=np.float32(c["bl"]),
        l8=q, vol0=vols[0], vol_sha=np.array([sha(v) for v in vols]),
        disp=np.stack([w[0] for w in wt]), conf=np.stack([w[1] for w in wt]), sad=sad)


if __name__ == "__main__":
    spixl_fixture()
    pixel_fixture()
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))
