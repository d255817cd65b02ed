"""Device-side stage API on torch tensors, backed by libmvs.so (HIP, gfx950).

torch supplies device memory, the HIP stream and ``torch.distributed``; every
compute step is a hand-written HIP kernel reached through the C-ABI in
include/mvs.h.  Tensors are in the reference layouts:

    rgbx   uint8   [V, H, W, 4]     lab    float32 [V, H, W, 4]
    spixl  float32 [V, mh, mw, 8]   labels int32   [V, H, W] (uint32 bits; the refinement
                                    and fusion also take 16-bit maps)
    rep    uint8   [V, mh, mw, 8]   state  float32 [V, mh, mw, 6]
    disp   float32 [V, H, W]
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from .params import map_size


def _ptr(t: torch.Tensor | None):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("libmvs device API needs CUDA (HIP) tensors")
    if not t.is_contiguous():
        raise ValueError("tensor must be contiguous")
    return C.c_void_p(t.data_ptr())


def _label_fn(L, name: str, labels: torch.Tensor):
    """The uint32 entry point `name`_d, or its 16-bit twin `name`_l16_d for
    int16/uint16 label maps (the narrowed all-gather's; bits read unsigned)."""
    if labels.dtype == torch.int32:
        return getattr(L, name + "_d")
    if labels.dtype in (torch.int16, torch.uint16):
        return getattr(L, name + "_l16_d")
    raise ValueError(f"labels must be int32 or 16-bit, not {labels.dtype}")


def _runs(views):
    """Sorted view ids -> contiguous [v0, v1) runs."""
    vs = sorted(set(int(v) for v in views))
    runs = []
    for v in vs:
        if runs and runs[-1][1] == v:
            runs[-1][1] = v + 1
        else:
            runs.append([v, v + 1])
    return [tuple(r) for r in runs]


@dataclass
class CameraArray:
    """Host-side camera-array metadata (pipeline::perform_depth_est)."""
    array_width: int
    bl_ratio: float
    levels: np.ndarray        # float32 [D]
    view_subset: np.ndarray   # int32 [V, V]
    subset_num: np.ndarray    # int32 [V]

    def __post_init__(self):
        self.levels = np.ascontiguousarray(self.levels, np.float32)
        self.view_subset = np.ascontiguousarray(self.view_subset, np.int32)
        self.subset_num = np.ascontiguousarray(self.subset_num, np.int32)
        self._desc = _lib.ArrayDesc(
            int(self.subset_num.shape[0]), int(self.array_width), float(self.bl_ratio),
            self.levels.ctypes.data_as(C.POINTER(C.c_float)), int(self.levels.shape[0]),
            self.view_subset.ctypes.data_as(C.POINTER(C.c_int32)),
            self.subset_num.ctypes.data_as(C.POINTER(C.c_int32)))

    @property
    def view_count(self) -> int:
        return int(self.subset_num.shape[0])

    @property
    def D(self) -> int:
        return int(self.levels.shape[0])

    def views_needed(self, z0: int, z1: int) -> list[int]:
        """Reference views [z0, z1) and every view their neighbour lists name:
        the views whose images a shard owning [z0, z1) reads."""
        need = set(range(z0, z1))
        for z in range(z0, z1):
            need.update(int(v) for v in self.view_subset[z, :int(self.subset_num[z])])
        return sorted(need)

    def desc(self):
        return C.byref(self._desc)


class Engine:
    """One libmvs context on one GPU (one process per GPU)."""

    def __init__(self, device: int = 0):
        self.L = _lib.load()
        if not torch.cuda.is_available():
            raise _lib.MvsError("no GPU visible: the MI355X engine has no CPU fallback")
        self.device = torch.device("cuda", device)
        ctx = C.c_void_p()
        _lib.check(self.L.mvs_create(device, C.byref(ctx)), "mvs_create")
        self.ctx = ctx
        self._levels_dev = {}

    def close(self):
        if self.ctx:
            self.L.mvs_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _stream(self):
        s = torch.cuda.current_stream(self.device).cuda_stream
        self.L.mvs_set_stream(self.ctx, C.c_void_p(s))

    def empty(self, shape, dtype):
        return torch.empty(shape, dtype=dtype, device=self.device)

    # ---- SLIC -------------------------------------------------------------
    def cvt(self, rgbx: torch.Tensor, want_l8: bool = True):
        V, H, W, _ = rgbx.shape
        lab = self.empty((V, H, W, 4), torch.float32)
        l8 = self.empty((V, H, W), torch.uint8) if want_l8 else None
        self._stream()
        _lib.check(self.L.mvs_cvt_d(self.ctx, _ptr(rgbx), V, W, H, _ptr(lab), _ptr(l8)), "mvs_cvt_d")
        return lab, l8

    def cvt_views(self, rgbx: torch.Tensor, views, lab: torch.Tensor, l8: torch.Tensor | None = None):
        """cvt of the listed views only, into full-size [V, ...] lab / l8 (a view
        shard converts its block and the block's neighbours)."""
        V, H, W, _ = rgbx.shape
        self._stream()
        for v0, v1 in _runs(views):
            _lib.check(self.L.mvs_cvt_d(self.ctx, _ptr(rgbx[v0:v1]), v1 - v0, W, H, _ptr(lab[v0:v1]),
                                        None if l8 is None else _ptr(l8[v0:v1])), "mvs_cvt_d")
        return lab, l8

    def slic(self, lab: torch.Tensor, S: int, weight: float = 0.6, no_iter: int = 5, enforce_connectivity=False,
             spixl=None, labels=None, edge_enable: int = 0, search: int = 0):
        """mvs_slic_d.  edge_enable (include/mvs.h): 0 off, 1 the reference's
        apply_edge_values as it behaves (overwrites `lab` in place), 2 the
        intended centre perturbation.  search: 0 the reference's active 2x2
        candidate loop, 1 the 3x3 loop behind its comment switch."""
        V, H, W, _ = lab.shape
        mw, mh = map_size(W, H, S)
        # s7 (disparity) is never written by the reference's SLIC (clcode.cl:285-293);
        # k_init_centers zeroes it, so every word of spixl is written
        spixl = self.empty((V, mh, mw, 8), torch.float32) if spixl is None else spixl
        labels = self.empty((V, H, W), torch.int32) if labels is None else labels
        if spixl.shape != (V, mh, mw, 8) or labels.shape != (V, H, W):
            raise ValueError("slic: output shapes do not match")
        p = _lib.SlicParams(int(S), float(weight), int(no_iter), int(bool(enforce_connectivity)), int(edge_enable),
                            int(search))
        self._stream()
        _lib.check(self.L.mvs_slic_d(self.ctx, _ptr(lab), V, W, H, C.byref(p), _ptr(spixl), _ptr(labels)),
                   "mvs_slic_d")
        return spixl, labels

    def grid(self, lab: torch.Tensor, S: int):
        V, H, W, _ = lab.shape
        mw, mh = map_size(W, H, S)
        spixl = self.empty((V, mh, mw, 8), torch.float32)  # every word written (s7 = 0)
        labels = self.empty((V, H, W), torch.int32)
        self._stream()
        _lib.check(self.L.mvs_grid_d(self.ctx, _ptr(lab), V, W, H, S, _ptr(spixl), _ptr(labels)), "mvs_grid_d")
        return spixl, labels

    # ---- photo-consistency ----------------------------------------------
    def boundary(self, spixl: torch.Tensor, labels: torch.Tensor, S: int):
        V, H, W = labels.shape
        mw, mh = map_size(W, H, S)
        rep = self.empty((V, mh, mw, 8), torch.uint8)
        self._stream()
        _lib.check(self.L.mvs_boundary_d(self.ctx, V, W, H, S, _ptr(spixl), _ptr(labels), _ptr(rep)),
                   "mvs_boundary_d")
        return rep

    def sweep_spixl(self, lab, spixl, rep, cam: CameraArray, S: int, z0: int = 0, z1: int | None = None):
        """initial_depth_estimation_v2 in place on spixl[..., 7]."""
        V, H, W, _ = lab.shape
        z1 = V if z1 is None else z1
        self._stream()
        _lib.check(self.L.mvs_sweep_spixl_d(self.ctx, W, H, S, _ptr(lab), _ptr(spixl), _ptr(rep), cam.desc(), z0, z1),
                   "mvs_sweep_spixl_d")
        return spixl

    def sweep_pixel_sad(self, lab, cam: CameraArray, z0: int = 0, z1: int | None = None, out=None):
        V, H, W, _ = lab.shape
        z1 = V if z1 is None else z1
        out = self.empty((z1 - z0, H, W), torch.float32) if out is None else out
        self._stream()
        _lib.check(self.L.mvs_sweep_pixel_sad_d(self.ctx, W, H, _ptr(lab), cam.desc(), z0, z1, _ptr(out)),
                   "mvs_sweep_pixel_sad_d")
        return out

    def box_stats(self, l8, K: int = 5, out=None):
        V, H, W = l8.shape
        # [0] window stats {S, bits(1/var | NaN)}, [1] packed intensities {lo, hi};
        # rows pairwise interleaved over Hp = H rounded up to even (include/mvs.h)
        out = self.empty((2, V, H + (H & 1), W, 2), torch.int32) if out is None else out
        self._stream()
        _lib.check(self.L.mvs_box_stats_d(self.ctx, _ptr(l8), V, W, H, K, _ptr(out)), "mvs_box_stats_d")
        return out

    def box_stats_views(self, l8, K: int, views, out):
        """Window planes of the listed views only, into a full V-view buffer."""
        V, H, W = l8.shape
        self._stream()
        for v0, v1 in _runs(views):
            _lib.check(self.L.mvs_box_stats_range_d(self.ctx, _ptr(l8), V, W, H, K, v0, v1, _ptr(out)),
                       "mvs_box_stats_range_d")
        return out

    def set_ncc_variant(self, waves: int = 0, levels_per_wave: int = 0, band_w: int = 0, general_rows: bool = False):
        """Force the NCC sweep variant tried first (0 = automatic; test / tuning hook)."""
        _lib.check(self.L.mvs_set_ncc_variant(self.ctx, int(waves), int(levels_per_wave), int(band_w),
                                              int(bool(general_rows))), "mvs_set_ncc_variant")

    def set_kernel_timing(self, on: bool) -> None:
        """Record start / stop events of every fused NCC sweep launch's own dispatch (bench aid)."""
        _lib.check(self.L.mvs_set_kernel_timing(self.ctx, int(bool(on))), "mvs_set_kernel_timing")

    def kernel_times(self, cap: int = 8192) -> list:
        """The recorded fused-sweep launches' kernel times in ms (waits for them; starts a new record)."""
        buf = (C.c_float * cap)()
        n = C.c_int(0)
        rc = self.L.mvs_kernel_times(self.ctx, buf, cap, C.byref(n))
        if rc != 0 and n.value > cap:
            return self.kernel_times(n.value)  # the record is kept: read it whole
        _lib.check(rc, "mvs_kernel_times")
        return list(buf[:n.value])

    def ncc_last_variant(self) -> dict:
        """The last NCC launch: K, tile rows, levels per wave, waves, band width,
        PAR (row parity: 0 mixed, 1 every band row pair-aligned, 2 odd pk / even
        stats rows), FUSE, NB (band buffers: 1 single, 2 double)."""
        v = (C.c_int32 * 8)()
        if self.L.mvs_ncc_last_variant_n(self.ctx, v, 8) != 8:
            raise _lib.MvsError("mvs_ncc_last_variant_n: unexpected slot count")
        return dict(zip(("K", "TH", "DPW", "NW", "BW", "PAR", "FUSE", "NB"), list(v)))

    def ncc_volume(self, l8, box, cam: CameraArray, z: int, K: int = 5, out=None):
        V, H, W = l8.shape
        out = self.empty((cam.D, H, W), torch.float32) if out is None else out
        self._stream()
        _lib.check(self.L.mvs_ncc_volume_d(self.ctx, W, H, _ptr(l8), _ptr(box), cam.desc(), K, z, _ptr(out)),
                   "mvs_ncc_volume_d")
        return out

    def ncc_wta(self, l8, box, cam: CameraArray, z: int, K: int = 5, disp=None, conf=None, want_conf: bool = True):
        """ncc_volume + wta in one kernel: the volume never reaches HBM (bit-identical)."""
        V, H, W = l8.shape
        disp = self.empty((H, W), torch.float32) if disp is None else disp
        if want_conf and conf is None:
            conf = self.empty((H, W), torch.float32)
        self._stream()
        _lib.check(self.L.mvs_ncc_wta_d(self.ctx, W, H, _ptr(l8), _ptr(box), cam.desc(), K, z, _ptr(disp),
                                        _ptr(conf) if want_conf else None), "mvs_ncc_wta_d")
        return disp, conf

    def ncc_wta_range(self, l8, box, cam: CameraArray, z0: int, z1: int, K: int = 5, disp=None, conf=None,
                      want_conf: bool = True):
        """ncc_wta for reference views [z0, z1) into disp/conf [z1 - z0, H, W]; views sharing a
        sweep variant go in one launch (bit-identical to one ncc_wta per view)."""
        V, H, W = l8.shape
        n = z1 - z0
        disp = self.empty((n, H, W), torch.float32) if disp is None else disp
        if want_conf and conf is None:
            conf = self.empty((n, H, W), torch.float32)
        for t in (disp, conf) if want_conf else (disp,):
            if tuple(t.shape) != (n, H, W) or not t.is_contiguous():
                raise ValueError("disp / conf must be contiguous [z1 - z0, H, W]")
        self._stream()
        _lib.check(self.L.mvs_ncc_wta_range_d(self.ctx, W, H, _ptr(l8), _ptr(box), cam.desc(), K, z0, z1,
                                              _ptr(disp), _ptr(conf) if want_conf else None),
                   "mvs_ncc_wta_range_d")
        return disp, conf

    def levels_dev(self, cam: CameraArray) -> torch.Tensor:
        key = cam.levels.tobytes()
        t = self._levels_dev.get(key)
        if t is None:
            t = torch.from_numpy(cam.levels.copy()).to(self.device)
            self._levels_dev[key] = t
        return t

    def wta(self, vol, levels: torch.Tensor, disp=None, conf=None, want_conf: bool = True):
        D, H, W = vol.shape
        disp = self.empty((H, W), torch.float32) if disp is None else disp
        if want_conf and conf is None:
            conf = self.empty((H, W), torch.float32)
        self._stream()
        _lib.check(self.L.mvs_wta_d(self.ctx, W, H, D, _ptr(vol), _ptr(levels), _ptr(disp),
                                    _ptr(conf) if want_conf else None), "mvs_wta_d")
        return disp, conf

    # ---- refinement ------------------------------------------------------
    def refine(self, spixl, labels, rep, cam: CameraArray, S: int, gamma=2.0, alpha=6.0, fuse=1.0, kernel_step=13,
               kernel_size=1080, no_prop=5, fusion_compat=True, want_disp=True):
        V, H, W = labels.shape
        mw, mh = map_size(W, H, S)
        flat = self.empty((V, mh, mw, 2), torch.float32)
        st = self.empty((V, mh, mw, 6), torch.float32)
        st2 = self.empty((V, mh, mw, 6), torch.float32)
        disp = self.empty((V, H, W), torch.float32) if want_disp else None
        p = _lib.RefineParams(float(gamma), float(alpha), float(fuse), int(kernel_step), int(kernel_size),
                              int(no_prop), int(bool(fusion_compat)))
        self._stream()
        _lib.check(self.L.mvs_refine_d(self.ctx, W, H, S, _ptr(spixl), _ptr(labels), _ptr(rep), cam.desc(),
                                       C.byref(p), _ptr(flat), _ptr(st), _ptr(st2), _ptr(disp)), "mvs_refine_d")
        final = st
        if not fusion_compat and no_prop > 0:
            final = st2 if (no_prop - 1) % 2 == 0 else st
        return {"flat": flat, "state": final, "state_compat": st, "disp": disp}

    def flatness(self, spixl, gamma: float):
        V, mh, mw, _ = spixl.shape
        flat = self.empty((V, mh, mw, 2), torch.float32)
        self._stream()
        _lib.check(self.L.mvs_flatness_d(self.ctx, V, mw, mh, _ptr(spixl), C.c_float(gamma), _ptr(flat)),
                   "mvs_flatness_d")
        return flat

    def init_state(self, spixl, labels, rep, flat, cam: CameraArray, S, gamma, alpha, nks, kss, fuse):
        V, H, W = labels.shape
        mw, mh = map_size(W, H, S)
        st = self.empty((V, mh, mw, 6), torch.float32)
        self._stream()
        _lib.check(self.L.mvs_init_state_d(self.ctx, W, H, S, _ptr(spixl), _ptr(labels), _ptr(rep), _ptr(flat),
                                           cam.desc(), C.c_float(gamma), C.c_float(alpha), int(nks), C.c_float(kss),
                                           C.c_float(fuse), _ptr(st)), "mvs_init_state_d")
        return st

    def init_state_range(self, spixl, labels, rep, flat, cam: CameraArray, S, gamma, alpha, nks, kss, fuse, z0, z1,
                         state=None):
        """init_current_state for views [z0, z1) into a full [V, mh, mw, 6] state.
        labels: int32, or int16/uint16 (16-bit maps, mw * mh <= 65536)."""
        V, H, W = labels.shape
        mw, mh = map_size(W, H, S)
        st = self.empty((V, mh, mw, 6), torch.float32) if state is None else state
        self._stream()
        fn = _label_fn(self.L, "mvs_init_state_range", labels)
        _lib.check(fn(self.ctx, W, H, S, _ptr(spixl), _ptr(labels), _ptr(rep), _ptr(flat),
                                                 cam.desc(), C.c_float(gamma), C.c_float(alpha), int(nks),
                                                 C.c_float(kss), C.c_float(fuse), int(z0), int(z1), _ptr(st)),
                   fn.__name__)
        return st

    def propagate(self, spixl, labels, rep, flat, cam: CameraArray, S, it, alpha, gamma, fuse, nks, kss, st_in,
                  st_out, z0=0, z1=None):
        V, H, W = labels.shape
        z1 = V if z1 is None else z1
        self._stream()
        fn = _label_fn(self.L, "mvs_propagate", labels)
        _lib.check(fn(self.ctx, W, H, S, _ptr(spixl), _ptr(labels), _ptr(rep), _ptr(flat),
                                          cam.desc(), int(it), C.c_float(alpha), C.c_float(gamma), C.c_float(fuse),
                                          int(nks), C.c_float(kss), _ptr(st_in), _ptr(st_out), int(z0), int(z1)),
                   fn.__name__)
        return st_out

    def spixl_to_image(self, spixl, labels, state, S):
        V, H, W = labels.shape
        disp = self.empty((V, H, W), torch.float32)
        self._stream()
        fn = _label_fn(self.L, "mvs_spixl_to_image", labels)
        _lib.check(fn(self.ctx, V, W, H, S, _ptr(spixl), _ptr(labels), _ptr(state), _ptr(disp)), fn.__name__)
        return disp

    def filter(self, disp_full, array_width: int, bl_ratio: float, fuse: float = 1.0, z0: int = 0, z1=None,
               out=None):
        V, H, W = disp_full.shape
        z1 = V if z1 is None else z1
        proj = self.empty((V, H, W), torch.float32)
        out = torch.zeros((V, H, W), dtype=torch.float32, device=self.device) if out is None else out
        self._stream()
        _lib.check(self.L.mvs_filter_d(self.ctx, V, W, H, int(array_width), C.c_float(bl_ratio), C.c_float(fuse),
                                       _ptr(disp_full), _ptr(proj), _ptr(out), int(z0), int(z1)), "mvs_filter_d")
        return proj, out

    def proj_inv(self, disp_full, array_width: int, bl_ratio: float, z0: int, z1: int, proj=None, rows=None,
                 band=False):
        """project_to_reference_inv for references [z0, z1) into proj[z0:z1] ([V, H, W]);
        rows=(y0, y1): image rows [y0, y1) only -- with band=True `proj` is that row
        band alone, [V, y1 - y0, W] (the buffer its all-gather fills)."""
        V, H, W = disp_full.shape
        if band:
            if rows is None or proj is None or tuple(proj.shape) != (V, rows[1] - rows[0], W):
                raise ValueError("band=True needs rows=(y0, y1) and proj of shape [V, y1 - y0, W]")
        proj = self.empty((V, H, W), torch.float32) if proj is None else proj
        self._stream()
        if rows is None:
            _lib.check(self.L.mvs_proj_inv_d(self.ctx, V, W, H, int(array_width), C.c_float(bl_ratio),
                                             _ptr(disp_full), _ptr(proj), int(z0), int(z1)), "mvs_proj_inv_d")
        else:
            _lib.check(self.L.mvs_proj_inv_rows_d(self.ctx, V, W, H, int(array_width), C.c_float(bl_ratio),
                                                  _ptr(disp_full), _ptr(proj), int(bool(band)), int(z0), int(z1),
                                                  int(rows[0]), int(rows[1])), "mvs_proj_inv_rows_d")
        return proj

    def remove_inconsistency(self, disp_full, proj, array_width: int, bl_ratio: float, fuse: float, z0: int, z1: int,
                             out=None, rows=None, band=False):
        """remove_view_inconsistency for references [z0, z1) (every proj slice filled; rows=(y0, y1):
        image rows [y0, y1) only, which read only those rows of proj -- with band=True `proj` is
        that row band alone, [V, y1 - y0, W])."""
        V, H, W = disp_full.shape
        out = torch.zeros((V, H, W), dtype=torch.float32, device=self.device) if out is None else out
        if band and (rows is None or tuple(proj.shape) != (V, rows[1] - rows[0], W)):
            raise ValueError("band=True needs rows=(y0, y1) and proj of shape [V, y1 - y0, W]")
        self._stream()
        if rows is None:
            _lib.check(self.L.mvs_remove_inconsistency_d(self.ctx, V, W, H, int(array_width), C.c_float(bl_ratio),
                                                         C.c_float(fuse), _ptr(disp_full), _ptr(proj), _ptr(out),
                                                         int(z0), int(z1)), "mvs_remove_inconsistency_d")
        else:
            _lib.check(self.L.mvs_remove_inconsistency_rows_d(self.ctx, V, W, H, int(array_width),
                                                              C.c_float(bl_ratio), C.c_float(fuse), _ptr(disp_full),
                                                              _ptr(proj), int(bool(band)), _ptr(out), int(z0), int(z1),
                                                              int(rows[0]), int(rows[1])),
                       "mvs_remove_inconsistency_rows_d")
        return out

    def synchronize(self):
        _lib.check(self.L.mvs_synchronize(self.ctx), "mvs_synchronize")
