"""Host-side parameter derivation, restating the reference's orchestration.

* ``disparity_levels``  <- pipeline::perform_depth_est, pipeline.cpp:121-124
* ``neighbour_lists``   <- pipeline::perform_depth_est, pipeline.cpp:130-142
* ``flatten_subsets``   <- clPhotoConsistency::do_initial_depth_estimation,
  photo_consistency.cpp:38-47 (V x V matrix, row z = neighbour list of z)
* ``Settings``          <- system_settings, header.h:55-77; defaults are the
  values main() hard-codes (clMVDE.cpp:14-36)
* SLIC / refinement scalar derivations <- clSLIC.cpp:15-22,
  depth_refinement.cpp:130, 335-339, 735-737, pipeline.cpp:164-166
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


@dataclass
class Settings:
    spixl_size: int = 8
    slic_color_weight: float = 0.6
    array_width: int = 3
    array_height: int = 3
    no_iter: int = 5
    enforce_connectivity: bool = False
    edge_enable: bool = False
    # find_center_association candidates: 0 the active 2x2 loop (clcode.cl:474-494),
    # 1 the 3x3 loop behind the reference's comment switch (clcode.cl:496-516)
    slic_search: int = 0
    num_disp_levels: int = 30
    neib_hor: int = 1
    neib_ver: int = 1
    min_disp: int = 30
    max_disp: int = 60
    inc: int = 1
    bl_ratio: float = 1.03590
    kernel_size: int = 1080
    kernel_step: int = 13
    fuse: float = 1.0
    gamma: float = 2.0
    alpha: float = 6.0
    no_prop: int = 5
    # build-defined extensions (no reference counterpart)
    cost: str = "sad"          # "sad" (reference parity) | "ncc"
    window: int = 5            # NCC window K (SAD parity is fixed at 5x5)
    extra: dict = field(default_factory=dict)

    @property
    def view_count(self) -> int:
        return self.array_width * self.array_height


def map_size(W: int, H: int, S: int) -> tuple[int, int]:
    """pipeline.cpp:18-19 -> (mw, mh)."""
    return int(math.ceil(float(np.float32(W) / np.float32(S)))), int(math.ceil(float(np.float32(H) / np.float32(S))))


def disparity_levels(min_disp: int, max_disp: int, inc: int) -> np.ndarray:
    return np.array([min_disp + i * inc for i in range((max_disp - min_disp) // inc + 1)], np.float32)


def neighbour_lists(array_width: int, array_height: int, neib_hor: int, neib_ver: int) -> list[list[int]]:
    V = array_width * array_height
    out: list[list[int]] = []
    for i in range(V):
        lst = []
        for x in range(i % array_width - neib_hor, i % array_width + neib_hor + 1):
            for y in range(i // array_width - neib_ver, i // array_width + neib_ver + 1):
                idx = y * array_width + x
                if 0 <= x < array_width and 0 <= y < array_height and idx != i:
                    lst.append(idx)
        out.append(lst)
    return out


def flatten_subsets(view_subset: list[list[int]]) -> tuple[np.ndarray, np.ndarray]:
    V = len(view_subset)
    mat = np.zeros((V, V), np.int32)
    num = np.zeros(V, np.int32)
    for i, lst in enumerate(view_subset):
        num[i] = len(lst)
        mat[i, :len(lst)] = lst
    return mat, num


def nearest_neighbours(array_width: int, array_height: int, k: int) -> list[list[int]]:
    """Explicit k-nearest neighbour lists (grid L2 distance, ties by index) used
    for large arrays (BASELINE config 4); not a reference code path."""
    V = array_width * array_height
    out = []
    for i in range(V):
        cx, cy = i % array_width, i // array_width
        cand = sorted((((v % array_width - cx) ** 2 + (v // array_width - cy) ** 2), v) for v in range(V) if v != i)
        out.append([v for _, v in cand[:k]])
    return out


def slic_normalisers(S: int) -> tuple[float, float]:
    """clSLIC ctor (clSLIC.cpp:15-18): (max_xy_dist, max_color_dist), float host maths."""
    f = np.float32
    xy = f(1.0) / (f(1.4242) * f(S))
    col = f(15.0) / (f(1.7321) * f(128))
    return float(f(xy * xy)), float(f(col * col))


def slic_grid(S: int, local: int = 16) -> tuple[int, int]:
    """(G = num_grid_per_center, cluster_per_line), clSLIC.cpp:20-21, 313."""
    G = int(math.ceil(float(np.float32(S * S * 9) / np.float32(local * local))))
    return G, (S * 3) // local


def refine_params(st: Settings) -> dict:
    """Scalars the refinement kernels receive (depth_refinement.cpp, pipeline.cpp:164-166)."""
    f = np.float32
    gamma_ = f(2 * float(st.gamma) ** 2)
    alpha_ = f(2 * float(st.alpha) ** 2)
    kernel_size = st.kernel_size // 2
    kss = f(max(1, kernel_size // st.kernel_step * st.spixl_size))
    return {
        "flat_gamma": float(f(1.0 / float(f(gamma_)))),
        "init_gamma": float(f(1) / gamma_),
        "init_alpha": float(f(1) / alpha_),
        "prop_gamma": float(f(1.0 / float(gamma_))),
        "prop_alpha": float(f(1.0 / float(alpha_))),
        "kernel_steps": st.kernel_step,
        "kss": float(kss),
        "fuse": float(f(0.5 * st.fuse)),
    }


def prop_schedule(iter_: int, kernel_steps: int, kss: float) -> tuple[int, float]:
    """depth_refinement.cpp:768-769: (no_kernel_steps/(iter+1), kss/(iter+1))."""
    return kernel_steps // (iter_ + 1), float(np.float32(kss) / np.float32(iter_ + 1))
