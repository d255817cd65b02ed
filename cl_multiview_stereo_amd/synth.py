"""Seeded synthetic camera-array stacks.

The reference ships only real photographs (Images/*) with no ground truth, so
tests and benchmarks use rendered stacks that follow the reference's own camera
model: view ``v`` sits at grid position ``(v % array_width, v // array_width)``
and a scene point with disparity ``d`` seen at ``(x, y)`` from the canonical
camera appears at ``(x - d*dx, y - bl_ratio*d*dy)`` in a view offset by
``(dx, dy)`` grid steps (photo_consistency kernel, clcode.cl:1033-1034).

Output images are packed exactly as the reference host packs them:
``[H][W][4]`` uint8 with s0=R, s1=G, s2=B, s3=0 (file_handler.cpp:6-14).
"""
from __future__ import annotations

import numpy as np


def _box3(img: np.ndarray) -> np.ndarray:
    p = np.pad(img.astype(np.int32), ((1, 1), (1, 1), (0, 0)), mode="edge")
    acc = np.zeros(img.shape, np.int32)
    for dy in range(3):
        for dx in range(3):
            acc += p[dy:dy + img.shape[0], dx:dx + img.shape[1]]
    return (acc // 9).astype(np.uint8)


def make_texture(W: int, H: int, rng: np.random.Generator) -> np.ndarray:
    """iid uniform RGB, 3x3 box blurred, plus 3-5 flat-coloured rectangles."""
    tex = _box3(rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8))
    for _ in range(int(rng.integers(3, 6))):
        w = int(rng.integers(max(2, W // 10), max(3, W // 3)))
        h = int(rng.integers(max(2, H // 10), max(3, H // 3)))
        x0 = int(rng.integers(0, max(1, W - w)))
        y0 = int(rng.integers(0, max(1, H - h)))
        tex[y0:y0 + h, x0:x0 + w] = rng.integers(0, 256, size=3, dtype=np.uint8)
    return tex


def make_disparity(W: int, H: int, dmin: int, dmax: int, rng: np.random.Generator) -> np.ndarray:
    """Piecewise fronto-parallel integer disparity planes in [dmin, dmax]."""
    disp = np.full((H, W), int(rng.integers(dmin, dmin + max(1, (dmax - dmin) // 4) + 1)), np.int32)
    for _ in range(int(rng.integers(2, 5))):
        w = int(rng.integers(max(2, W // 8), max(3, W // 2)))
        h = int(rng.integers(max(2, H // 8), max(3, H // 2)))
        x0 = int(rng.integers(0, max(1, W - w)))
        y0 = int(rng.integers(0, max(1, H - h)))
        disp[y0:y0 + h, x0:x0 + w] = int(rng.integers(dmin, dmax + 1))
    return disp


def render_stack(tex: np.ndarray, disp: np.ndarray, array_width: int, array_height: int,
                 bl_ratio: float, rng: np.random.Generator, centre: tuple[float, float] | None = None) -> np.ndarray:
    """Forward-splat the canonical texture into every view (z-buffer: larger d wins)."""
    H, W, _ = tex.shape
    V = array_width * array_height
    cx0, cy0 = centre if centre is not None else ((array_width - 1) / 2.0, (array_height - 1) / 2.0)
    ys, xs = np.mgrid[0:H, 0:W]
    out = np.zeros((V, H, W, 4), np.uint8)
    for v in range(V):
        vx, vy = v % array_width, v // array_width
        tx = np.rint(xs - disp * (vx - cx0)).astype(np.int64)
        ty = np.rint(ys - bl_ratio * disp * (vy - cy0)).astype(np.int64)
        ok = (tx >= 0) & (tx < W) & (ty >= 0) & (ty < H)
        flat = (ty * W + tx)[ok]
        dd = disp[ok]
        # z-buffer (max disparity per target pixel): scatter the few distinct
        # disparities in increasing order, so the largest lands last
        z = np.full(H * W, -1, np.int64)
        for dv in np.unique(dd):
            z[flat[dd == dv]] = dv
        win = dd == z[flat]
        img = rng.integers(0, 256, size=(H * W, 3), dtype=np.uint8)  # holes -> noise
        img[flat[win]] = tex.reshape(-1, 3)[np.flatnonzero(ok)[win]]
        out[v, :, :, :3] = img.reshape(H, W, 3)
    return out


def make_stack(W: int, H: int, array_width: int, array_height: int = 1, dmin: int = 0,
               dmax: int = 31, bl_ratio: float = 1.0, seed: int = 0x5EED):
    """Return (rgbx[V][H][W][4] uint8, canonical disparity[H][W] int32)."""
    rng = np.random.default_rng(seed)
    tex = make_texture(W, H, rng)
    disp = make_disparity(W, H, dmin, dmax, rng)
    # keep the disparity span inside what the sweep searches
    disp = np.clip(disp, dmin, dmax)
    stack = render_stack(tex, disp, array_width, array_height, bl_ratio, rng)
    return stack, disp


def random_stack(V: int, W: int, H: int, seed: int) -> np.ndarray:
    """Unstructured uint8 RGBx views (edge-case tests)."""
    rng = np.random.default_rng(seed)
    out = rng.integers(0, 256, size=(V, H, W, 4), dtype=np.uint8)
    out[..., 3] = 0
    return out
