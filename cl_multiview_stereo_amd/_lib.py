"""ctypes binding of libmvs.so (include/mvs.h).

The product path: every compute call goes through the HIP library.  There is
no CPU fallback -- if libmvs.so is missing or no GPU is visible, calls raise.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MVS_LIB: an alternative build of the same library (A/B timing of kernel variants)
LIB_PATH = os.environ.get("MVS_LIB") or os.path.join(_HERE, "libmvs.so")

# every symbol include/mvs.h declares (checked by tests/test_boundary.py)
EXPORTS = [
    "mvs_create", "mvs_destroy", "mvs_last_error", "mvs_set_stream", "mvs_synchronize", "mvs_version",
    "mvs_cvt_d", "mvs_slic_d", "mvs_grid_d", "mvs_boundary_d", "mvs_sweep_spixl_d", "mvs_sweep_pixel_sad_d",
    "mvs_box_stats_d", "mvs_ncc_volume_d", "mvs_wta_d", "mvs_ncc_wta_d", "mvs_ncc_wta_range_d", "mvs_flatness_d", "mvs_init_state_d",
    "mvs_propagate_d", "mvs_spixl_to_image_d", "mvs_refine_d", "mvs_filter_d",
    "mvs_box_stats_range_d", "mvs_set_ncc_variant", "mvs_ncc_last_variant", "mvs_ncc_last_variant_n", "mvs_set_kernel_timing", "mvs_kernel_times", "mvs_init_state_range_d",
    "mvs_proj_inv_d", "mvs_remove_inconsistency_d", "mvs_proj_inv_rows_d", "mvs_remove_inconsistency_rows_d",
    "mvs_do_super_pixel_seg", "mvs_do_initial_depth_estimation", "mvs_do_refinement", "mvs_do_consistency_filter",
    "mvs_init_state_range_l16_d", "mvs_propagate_l16_d", "mvs_spixl_to_image_l16_d",
]


class MvsError(RuntimeError):
    pass


class SlicParams(C.Structure):
    """mvs_slic_params (ABI 0.3): struct_size is filled in by the constructor."""
    _fields_ = [("struct_size", C.c_uint32), ("spixl_size", C.c_int), ("color_weight", C.c_float),
                ("no_iter", C.c_int), ("enforce_connectivity", C.c_int), ("edge_enable", C.c_int),
                ("search", C.c_int)]

    def __init__(self, spixl_size=8, color_weight=0.6, no_iter=5, enforce_connectivity=0, edge_enable=0, search=0):
        super().__init__(C.sizeof(SlicParams), spixl_size, color_weight, no_iter, enforce_connectivity,
                         edge_enable, search)


class ArrayDesc(C.Structure):
    _fields_ = [("view_count", C.c_int), ("array_width", C.c_int), ("bl_ratio", C.c_float),
                ("levels", C.POINTER(C.c_float)), ("num_levels", C.c_int),
                ("view_subset", C.POINTER(C.c_int32)), ("subset_num", C.POINTER(C.c_int32))]


class RefineParams(C.Structure):
    """mvs_refine_params (ABI 0.3): struct_size is filled in by the constructor."""
    _fields_ = [("struct_size", C.c_uint32), ("gamma", C.c_float), ("alpha", C.c_float), ("fuse", C.c_float),
                ("kernel_step", C.c_int), ("kernel_size", C.c_int), ("no_prop", C.c_int),
                ("fusion_compat", C.c_int), ("prescaled", C.c_int)]

    def __init__(self, gamma=2.0, alpha=6.0, fuse=1.0, kernel_step=13, kernel_size=1080, no_prop=5,
                 fusion_compat=1, prescaled=0):
        super().__init__(C.sizeof(RefineParams), gamma, alpha, fuse, kernel_step, kernel_size, no_prop,
                         fusion_compat, prescaled)


_lib = None


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load libmvs.so (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise MvsError(f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(path)
    L.mvs_last_error.restype = C.c_char_p
    L.mvs_version.restype = C.c_char_p
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        raise MvsError(f"{what} failed ({rc}): {load().mvs_last_error().decode()}")
