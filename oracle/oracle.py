"""ORACLE TEST INFRASTRUCTURE -- ctypes front-end of oracle/_build/liboracle.so.

CPU restatement of the reference hot path (oracle/mvs_oracle.c, pinned by the
reference's kept outputs -- see that file's header and DESIGN.md 0).  MVS_ORACLE_LIB
selects another build of the same source (the ASan build: scripts/oracle_asan.sh).
Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg use it, and only as the checker / CPU baseline.
Every function takes and returns numpy arrays in the reference layouts.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MVS_ORACLE_LIB") or os.path.join(_HERE, "_build", "liboracle.so")
_lib = None

f32p = C.POINTER(C.c_float)
u8p = C.POINTER(C.c_uint8)
u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int32)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t)


def _f(x):
    return C.c_float(float(x))


def map_size(W, H, S):
    return lib().orc_map_w(W, S), lib().orc_map_h(H, S)


def cvt(rgbx):
    rgbx = np.ascontiguousarray(rgbx, np.uint8)
    H, W = rgbx.shape[-3:-1]
    n = rgbx.size // (4 * H * W)
    out = np.zeros(rgbx.shape[:-1] + (4,), np.float32)
    for v in range(n):
        src = rgbx.reshape(n, H, W, 4)[v]
        dst = out.reshape(n, H, W, 4)[v]
        lib().orc_cvt(_p(np.ascontiguousarray(src), u8p), W, H, _p(dst, f32p))
    return out


def l8(lab):
    lab = np.ascontiguousarray(lab, np.float32)
    H, W = lab.shape[-3:-1]
    n = lab.size // (4 * H * W)
    out = np.zeros(lab.shape[:-1], np.uint8)
    for v in range(n):
        src = np.ascontiguousarray(lab.reshape(n, H, W, 4)[v])
        dst = out.reshape(n, H, W)[v]
        lib().orc_l8(_p(src, f32p), W, H, _p(dst, u8p))
    return out


def slic(rgbx, S, weight=0.6, no_iter=5, enforce_connectivity=False, edge_enable=0, search=0):
    """clSLIC::do_super_pixel_seg for ONE view -> (lab, spixl, labels).
    edge_enable: 0 off, 1 the reference's apply_edge_values as it behaves
    (Lab overwritten by the edge magnitude), 2 the intended form (centres moved
    to the least-edge neighbour); orc_edge_step."""
    rgbx = np.ascontiguousarray(rgbx, np.uint8)
    H, W = rgbx.shape[:2]
    mw, mh = map_size(W, H, S)
    lab = np.zeros((H, W, 4), np.float32)
    sp = np.zeros((mh, mw, 8), np.float32)
    lb = np.zeros((H, W), np.uint32)
    lib().orc_slic_ex(_p(rgbx, u8p), W, H, S, _f(weight), no_iter, int(bool(enforce_connectivity)),
                      int(edge_enable), int(search), _p(lab, f32p), _p(sp, f32p), _p(lb, u32p))
    return lab, sp, lb


def edge(lab):
    """edge_compute_alternative magnitude [H][W] of ONE view (orc_edge)."""
    lab = np.ascontiguousarray(lab, np.float32)
    H, W = lab.shape[:2]
    out = np.zeros((H, W), np.float32)
    lib().orc_edge(_p(lab, f32p), W, H, _p(out, f32p))
    return out


def init_centers(lab, S):
    lab = np.ascontiguousarray(lab, np.float32)
    H, W = lab.shape[:2]
    mw, mh = map_size(W, H, S)
    sp = np.zeros((mh, mw, 8), np.float32)
    lib().orc_init_centers(_p(lab, f32p), W, H, S, _p(sp, f32p))
    return sp


def assign(lab, spixl, S, weight=0.6, search=0):
    lab = np.ascontiguousarray(lab, np.float32)
    spixl = np.ascontiguousarray(spixl, np.float32)
    H, W = lab.shape[:2]
    f = np.float32
    xy = f(1.0) / (f(1.4242) * f(S))
    col = f(15.0) / (f(1.7321) * f(128.0))
    lb = np.zeros((H, W), np.uint32)
    lib().orc_assign_ex(_p(lab, f32p), _p(spixl, f32p), W, H, S, _f(xy * xy), _f(col * col), _f(weight), int(search),
                        _p(lb, u32p))
    return lb


def update(lab, labels, S, spixl=None):
    lab = np.ascontiguousarray(lab, np.float32)
    labels = np.ascontiguousarray(labels, np.uint32)
    H, W = lab.shape[:2]
    mw, mh = map_size(W, H, S)
    sp = np.zeros((mh, mw, 8), np.float32) if spixl is None else np.array(spixl, np.float32, copy=True)
    lib().orc_update(_p(lab, f32p), _p(labels, u32p), W, H, S, _p(sp, f32p))
    return sp


def grid(rgbx, S):
    rgbx = np.ascontiguousarray(rgbx, np.uint8)
    H, W = rgbx.shape[:2]
    mw, mh = map_size(W, H, S)
    lab = np.zeros((H, W, 4), np.float32)
    sp = np.zeros((mh, mw, 8), np.float32)
    lb = np.zeros((H, W), np.uint32)
    lib().orc_grid(_p(rgbx, u8p), W, H, S, _p(lab, f32p), _p(sp, f32p), _p(lb, u32p))
    return lab, sp, lb


def boundary(spixl, labels, S):
    spixl = np.ascontiguousarray(spixl, np.float32)
    labels = np.ascontiguousarray(labels, np.uint32)
    V, H, W = labels.shape
    mw, mh = map_size(W, H, S)
    rep = np.zeros((V, mh, mw, 8), np.uint8)
    lib().orc_boundary(V, W, H, S, _p(spixl, f32p), _p(labels, u32p), _p(rep, u8p))
    return rep


def sweep(lab, spixl, rep, levels, view_subset, subset_num, array_width, bl_ratio, S, z0=0, z1=None):
    lab = np.ascontiguousarray(lab, np.float32)
    sp = np.array(spixl, np.float32, copy=True, order="C")
    rep = np.ascontiguousarray(rep, np.uint8)
    levels = np.ascontiguousarray(levels, np.float32)
    vs = np.ascontiguousarray(view_subset, np.int32)
    sn = np.ascontiguousarray(subset_num, np.int32)
    V, H, W = lab.shape[:3]
    z1 = V if z1 is None else z1
    lib().orc_sweep(V, W, H, S, _p(lab, f32p), _p(sp, f32p), _p(rep, u8p), _p(levels, f32p), len(levels),
                    _p(vs, i32p), _p(sn, i32p), array_width, _f(bl_ratio), z0, z1)
    return sp


def sweep_pixel_sad(lab, levels, view_subset, subset_num, array_width, bl_ratio, z0=0, z1=None):
    """initial_depth_estimation_v2 on the S=1 grid -> disp [z1-z0, H, W]."""
    V, H, W = lab.shape[:3]
    z1 = V if z1 is None else z1
    sps, lbs = [], []
    for v in range(V):
        sp = np.zeros((H, W, 8), np.float32)
        lib().orc_init_centers(_p(np.ascontiguousarray(lab[v]), f32p), W, H, 1, _p(sp, f32p))
        sps.append(sp)
    sp = np.stack(sps)
    rep = np.zeros((V, H, W, 8), np.uint8)
    out = sweep(lab, sp, rep, levels, view_subset, subset_num, array_width, bl_ratio, 1, z0, z1)
    return out[z0:z1, :, :, 7].copy()


def ncc_volume(l8_all, levels, view_subset, subset_num, array_width, bl_ratio, K, z):
    q = np.ascontiguousarray(l8_all, np.uint8)
    levels = np.ascontiguousarray(levels, np.float32)
    vs = np.ascontiguousarray(view_subset, np.int32)
    sn = np.ascontiguousarray(subset_num, np.int32)
    V, H, W = q.shape
    vol = np.zeros((len(levels), H, W), np.float32)
    lib().orc_ncc_volume(V, W, H, _p(q, u8p), _p(levels, f32p), len(levels), _p(vs, i32p), _p(sn, i32p),
                         array_width, _f(bl_ratio), K, z, _p(vol, f32p))
    return vol


def ncc_volume_f32(lab_all, levels, view_subset, subset_num, array_width, bl_ratio, K, z):
    """The NCC cost on the float L plane (no 8-bit quantisation, double sums):
    the accuracy yardstick of the i8 definition (scripts/ncc_i8_vs_f32.py)."""
    lab = np.ascontiguousarray(lab_all, np.float32)
    levels = np.ascontiguousarray(levels, np.float32)
    vs = np.ascontiguousarray(view_subset, np.int32)
    sn = np.ascontiguousarray(subset_num, np.int32)
    V, H, W = lab.shape[:3]
    vol = np.zeros((len(levels), H, W), np.float32)
    lib().orc_ncc_volume_f32(V, W, H, _p(lab, f32p), _p(levels, f32p), len(levels), _p(vs, i32p), _p(sn, i32p),
                             array_width, _f(bl_ratio), K, z, _p(vol, f32p))
    return vol


def wta(vol, levels):
    vol = np.ascontiguousarray(vol, np.float32)
    levels = np.ascontiguousarray(levels, np.float32)
    D, H, W = vol.shape
    disp = np.zeros((H, W), np.float32)
    conf = np.zeros((H, W), np.float32)
    lib().orc_wta(W, H, D, _p(vol, f32p), _p(levels, f32p), _p(disp, f32p), _p(conf, f32p))
    return disp, conf


def refine(spixl, labels, rep, view_subset, subset_num, array_width, bl_ratio, S, gamma=2.0, alpha=6.0, fuse=1.0,
           kernel_step=13, kernel_size=1080, no_prop=5, fusion_compat=True):
    spixl = np.ascontiguousarray(spixl, np.float32)
    labels = np.ascontiguousarray(labels, np.uint32)
    rep = np.ascontiguousarray(rep, np.uint8)
    vs = np.ascontiguousarray(view_subset, np.int32)
    sn = np.ascontiguousarray(subset_num, np.int32)
    V, H, W = labels.shape
    mw, mh = map_size(W, H, S)
    flat = np.zeros((V, mh, mw, 2), np.float32)
    st0 = np.zeros((V, mh, mw, 6), np.float32)
    sts = np.zeros((max(no_prop, 1), V, mh, mw, 6), np.float32)
    disp = np.zeros((V, H, W), np.float32)
    lib().orc_refine(V, W, H, S, array_width, _f(bl_ratio), _p(spixl, f32p), _p(labels, u32p), _p(rep, u8p),
                     _p(vs, i32p), _p(sn, i32p), _f(gamma), _f(alpha), _f(fuse), kernel_step, kernel_size, no_prop,
                     int(bool(fusion_compat)), _p(flat, f32p), _p(st0, f32p), _p(sts, f32p), _p(disp, f32p))
    return {"flat": flat, "state0": st0, "states": sts[:no_prop], "disp": disp}


def propagate(spixl, labels, rep, flat, view_subset, subset_num, array_width, bl_ratio, S, it, alpha, gamma, fuse,
              nks, kss, st_in, z0=0, z1=None):
    spixl = np.ascontiguousarray(spixl, np.float32)
    labels = np.ascontiguousarray(labels, np.uint32)
    rep = np.ascontiguousarray(rep, np.uint8)
    flat = np.ascontiguousarray(flat, np.float32)
    vs = np.ascontiguousarray(view_subset, np.int32)
    sn = np.ascontiguousarray(subset_num, np.int32)
    st_in = np.ascontiguousarray(st_in, np.float32)
    V, H, W = labels.shape
    z1 = V if z1 is None else z1
    out = st_in.copy()
    lib().orc_propagate(V, W, H, S, array_width, _f(bl_ratio), _p(spixl, f32p), _p(labels, u32p), _p(rep, u8p),
                        _p(flat, f32p), _p(vs, i32p), _p(sn, i32p), it, _f(alpha), _f(gamma), _f(fuse), nks,
                        _f(kss), _p(st_in, f32p), _p(out, f32p), z0, z1)
    return out


def spixl_to_image(spixl, labels, state, S):
    spixl = np.ascontiguousarray(spixl, np.float32)
    labels = np.ascontiguousarray(labels, np.uint32)
    state = np.ascontiguousarray(state, np.float32)
    V, H, W = labels.shape
    disp = np.zeros((V, H, W), np.float32)
    lib().orc_spixl_to_image(V, W, H, S, _p(spixl, f32p), _p(labels, u32p), _p(state, f32p), _p(disp, f32p))
    return disp


def filt(disp_full, array_width, bl_ratio, fuse=1.0):
    df = np.ascontiguousarray(disp_full, np.float32)
    V, H, W = df.shape
    proj = np.zeros_like(df)
    out = np.zeros_like(df)
    lib().orc_filter(V, W, H, array_width, _f(bl_ratio), _f(0.5 * fuse), _p(df, f32p), _p(proj, f32p),
                     _p(out, f32p))
    return proj, out


def flatness(spixl, gamma):
    spixl = np.ascontiguousarray(spixl, np.float32)
    V, mh, mw, _ = spixl.shape
    flat = np.zeros((V, mh, mw, 2), np.float32)
    lib().orc_flatness(V, mw, mh, _p(spixl, f32p), _f(gamma), _p(flat, f32p))
    return flat


def init_state(spixl, labels, rep, flat, view_subset, subset_num, array_width, bl_ratio, S, gamma, alpha, nks, kss,
               fuse):
    """init_current_state with the kernel-side scalars (1/gamma', 1/alpha', fuse/2)."""
    spixl = np.ascontiguousarray(spixl, np.float32)
    labels = np.ascontiguousarray(labels, np.uint32)
    rep = np.ascontiguousarray(rep, np.uint8)
    flat = np.ascontiguousarray(flat, np.float32)
    vs = np.ascontiguousarray(view_subset, np.int32)
    sn = np.ascontiguousarray(subset_num, np.int32)
    V, H, W = labels.shape
    mw, mh = map_size(W, H, S)
    st = np.zeros((V, mh, mw, 6), np.float32)
    lib().orc_init_state(V, W, H, S, array_width, _f(bl_ratio), _p(spixl, f32p), _p(labels, u32p), _p(rep, u8p),
                         _p(flat, f32p), _p(vs, i32p), _p(sn, i32p), _f(gamma), _f(alpha), int(nks), _f(kss),
                         _f(fuse), _p(st, f32p))
    return st


def suppress(labels):
    """supress_local_lable, one pass."""
    labels = np.ascontiguousarray(labels, np.uint32)
    H, W = labels.shape
    out = np.zeros_like(labels)
    lib().orc_suppress(_p(labels, u32p), _p(out, u32p), W, H)
    return out


def slic_from_lab(lab, S, weight=0.6, no_iter=5, enforce_connectivity=False, search=0):
    """clSLIC::do_super_pixel_seg minus its cvt, on one view's Lab."""
    sp = init_centers(lab, S)
    lb = assign(lab, sp, S, weight, search)
    for _ in range(no_iter):
        sp = update(lab, lb, S)
        lb = assign(lab, sp, S, weight, search)
    if enforce_connectivity:
        lb = suppress(suppress(lb))
    return sp, lb
