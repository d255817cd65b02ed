"""Second, independent restatement of the hot path in vectorised numpy.

Test infrastructure only.  It is written from the reference kernels
(clcode.cl, file:line per function) separately from oracle/mvs_oracle.c, and
the CPU suite checks the two against each other bit-for-bit (every step is an
elementwise IEEE f32 op in the same order, so numpy and gcc -ffp-contract=off
must agree exactly).  This is what keeps a slip in the C oracle from silently
becoming the GPU's definition of "correct".
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def map_size(W, H, S):
    return int(np.ceil(f32(W) / f32(S))), int(np.ceil(f32(H) / f32(S)))


def roundf(x):
    """C roundf (half away from zero) of float32 x, exact via float64."""
    x = np.asarray(x, np.float64)
    return np.trunc(x + np.copysign(0.5, x)).astype(np.int64)


def l8(lab):
    """Build-defined NCC intensity: clamp(int(L*2.55f + 0.5f))."""
    t = lab[..., 0].astype(f32) * f32(2.55)
    t = t + f32(0.5)
    return np.clip(np.trunc(t), 0, 255).astype(np.uint8)


def cvt_f64(rgbx):
    """rgb2lab (clcode.cl:21-59) in float64 with true cube roots; s0 read as blue."""
    c = rgbx[..., :3].astype(np.float64) * 0.0039216
    b, g, r = c[..., 0], c[..., 1], c[..., 2]
    x = r * 0.412453 + g * 0.357580 + b * 0.180423
    y = r * 0.212671 + g * 0.715160 + b * 0.072169
    z = r * 0.019334 + g * 0.119193 + b * 0.950227
    xr, yr, zr = x / 0.950456, y, z / 1.088754

    def f(t):
        return np.where(t > 0.008856, np.cbrt(t), (903.3 * t + 16.0) / 116.0)

    fx, fy, fz = f(xr), f(yr), f(zr)
    return np.stack([116.0 * fy - 16.0, 500.0 * (fx - fy), 200.0 * (fy - fz)], -1)


def grid_labels(W, H, S):
    """init_label_per_pixl, clcode.cl:341-353."""
    mw, _ = map_size(W, H, S)
    y, x = np.mgrid[0:H, 0:W]
    return (mw * (y // S) + x // S).astype(np.uint32)


def assign(lab, spixl, S, weight=0.6):
    """find_center_association + slic_distance_function, clcode.cl:422-520.
    The candidate loop runs i over the x delta and j over the y delta but
    offsets (cx + j, cy + i) -- the reference's swap."""
    H, W = lab.shape[:2]
    mw, mh = map_size(W, H, S)
    xy = f32(1.0) / (f32(1.4242) * f32(S))
    col = f32(15.0) / (f32(1.7321) * f32(128.0))
    sn, cn, wt = f32(xy * xy), f32(col * col), f32(weight)
    row, colx = np.mgrid[0:H, 0:W]
    cxg, cyg = colx // S, row // S
    dX = (colx + S // 2) // S - cxg
    dY = (row + S // 2) // S - cyg
    best = np.full((H, W), f32(999999.9999), f32)
    lbl = np.full((H, W), -1, np.int64)
    sp = spixl.reshape(-1, 8)
    fx, fy = colx.astype(f32), row.astype(f32)
    for di in (-1, 0):
        for dj in (-1, 0):
            i, j = di + dX, dj + dY
            cx, cy = cxg + j, cyg + i
            ok = (cx >= 0) & (cy >= 0) & (cx < mw) & (cy < mh)
            ci = np.where(ok, cy * mw + cx, 0)
            c = sp[ci]
            a = (lab[..., 0] - c[..., 3]) * (lab[..., 0] - c[..., 3])
            a = a + (lab[..., 1] - c[..., 4]) * (lab[..., 1] - c[..., 4])
            a = a + (lab[..., 2] - c[..., 5]) * (lab[..., 2] - c[..., 5])
            b = (fx - c[..., 1]) * (fx - c[..., 1])
            b = b + (fy - c[..., 2]) * (fy - c[..., 2])
            d = np.sqrt((a * cn) + wt * (b * sn)).astype(f32)
            take = ok & (d < best)
            best = np.where(take, d, best)
            lbl = np.where(take, ci, lbl)
    return lbl.astype(np.uint32)


def update(lab, labels, S, local=16):
    """update_cluster_center + finalize_reduction_result, clcode.cl:533-611, 719-773:
    per (superpixel, 16x16 tile) the LDS tree v[k] += v[k+i], i = 128..1, then
    the tile partials summed in tile order and divided by the count."""
    H, W = lab.shape[:2]
    mw, mh = map_size(W, H, S)
    M = mw * mh
    G = int(np.ceil(f32(S * S * 9) / f32(local * local)))
    cpl = S * 3 // local
    sp = np.arange(M)
    gx, gy = sp % mw, sp // mw
    ly, lx = np.divmod(np.arange(local * local), local)
    acc = np.zeros((M, 6), f32)
    for t in range(G):
        nbx, nby = t % cpl, t // cpl
        pxo, pyo = nbx * local + lx, nby * local + ly
        px = gx[:, None] * S - S + pxo[None, :]
        py = gy[:, None] * S - S + pyo[None, :]
        ok = (pyo < 3 * S)[None, :] & (pxo < 3 * S)[None, :] & (py >= 0) & (px >= 0) & (px < W) & (py < H)
        pi = np.where(ok, py * W + px, 0)
        ok &= labels.reshape(-1)[pi] == sp[:, None]
        L = lab.reshape(-1, 4)[pi]
        v = np.zeros((M, 256, 6), f32)
        v[..., 0] = np.where(ok, px, 0)
        v[..., 1] = np.where(ok, py, 0)
        for c in range(3):
            v[..., 2 + c] = np.where(ok, L[..., c], 0)
        v[..., 5] = ok
        i = 128
        while i:
            v[:, :i] = v[:, :i] + v[:, i:2 * i]
            i //= 2
        acc = acc + v[:, 0]
    out = np.zeros((M, 8), f32)
    out[:, 0] = sp
    n = acc[:, 5]
    nz = n != 0
    for c in range(5):
        out[nz, 1 + c] = acc[nz, c] * (f32(1) / n[nz])  # x * RN(1/n): DESIGN.md section 0
    out[nz, 6] = n[nz]
    return out.reshape(mh, mw, 8)


def suppress(lbl):
    """supress_local_lable, clcode.cl:676-711: a pixel with >= 16 differing
    labels in its 5x5 takes the LAST differing one (row-major scan)."""
    H, W = lbl.shape
    out = lbl.copy()
    src = lbl.astype(np.int64)
    cnt = np.zeros((H - 4, W - 4), np.int64)
    last = np.full((H - 4, W - 4), -1, np.int64)
    c = src[2:H - 2, 2:W - 2]
    for j in range(-2, 3):
        for i in range(-2, 3):
            nl = src[2 + j:H - 2 + j, 2 + i:W - 2 + i]
            diff = nl != c
            cnt += diff
            last = np.where(diff, nl, last)
    out[2:H - 2, 2:W - 2] = np.where(cnt >= 16, last, c).astype(np.uint32)
    return out


def boundary(spixl, labels, S):
    """find_super_pixel_boundary, clcode.cl:791-855 -> rep [V][mh][mw][8]."""
    V, H, W = labels.shape
    mw, mh = map_size(W, H, S)
    rep = np.zeros((V, mh, mw, 8), np.uint8)
    dirs = [(-1, -1), (-1, 0), (-1, 1), (0, -1), (0, 1), (1, -1), (1, 0), (1, 1)]  # (sx, sy)
    for z in range(V):
        for ty in range(mh):
            for tx in range(mw):
                s = spixl[z, ty, tx]
                cx, cy = int(s[1]), int(s[2])
                if cx < S:
                    cx += S - cx
                if cx + S > W:
                    cx -= S
                if cy < S:
                    cy += S - cy
                if cy + S > H:
                    cy -= S
                sid = ty * mw + tx
                for k, (sx, sy) in enumerate(dirs):
                    for i in range(1, S):
                        x, y = cx + sx * i, cy + sy * i
                        if 0 <= x < W and 0 <= y < H and labels[z, y, x] == sid:
                            rep[z, ty, tx, k] = i - 1
    return rep


def sweep_pixel_sad(lab, levels, vs, sn, aw, bl):
    """initial_depth_estimation_v2 (clcode.cl:972-1069) on the S=1 grid: every
    pixel is a superpixel centre with unit ray steps.  The tap sequence
    val += 30; (valid) val -= 30, val += AD is kept op for op."""
    V, H, W = lab.shape[:3]
    bl = f32(bl)
    y, x = np.mgrid[0:H, 0:W]
    out = np.zeros((V, H, W), f32)
    for z in range(V):
        rx, ry = z % aw, z // aw
        cost = np.full((H, W), f32(1e6), f32)
        disp = np.zeros((H, W), f32)
        for d in np.asarray(levels, f32):
            mn = np.full((H, W), f32(1e6), f32)
            for n in range(sn[z]):
                view = vs[z, n]
                dxv, dyv = f32(view % aw - rx), f32(view // aw - ry)
                val = np.zeros((H, W), f32)
                for i in range(-2, 3):
                    for j in range(-2, 3):
                        xr, yr = x + i, y + j
                        xp = np.trunc(xr.astype(f32) - d * dxv).astype(np.int64)
                        yp = np.trunc(yr.astype(f32) - (bl * d) * dyv).astype(np.int64)
                        val = val + f32(30)
                        ok = (xr >= 0) & (yr >= 0) & (xp >= 0) & (yp >= 0) & (xr < W) & (yr < H) & (xp < W) & (yp < H)
                        a = lab[z, np.clip(yr, 0, H - 1), np.clip(xr, 0, W - 1)]
                        b = lab[view, np.clip(yp, 0, H - 1), np.clip(xp, 0, W - 1)]
                        ad = np.abs(a[..., 0] - b[..., 0]) + np.abs(a[..., 1] - b[..., 1])
                        ad = ad + np.abs(a[..., 2] - b[..., 2])
                        val = np.where(ok, (val - f32(30)) + ad, val)
                mn = np.where(val < mn, val, mn)
            take = mn < cost
            cost = np.where(take, mn, cost)
            disp = np.where(take, d, disp)
        out[z] = disp
    return out


def _box(a, r):
    """Integer K x K window sums (valid region only) of a [H][W] int64 array."""
    H, W = a.shape
    c = np.zeros((H + 1, W + 1), np.int64)
    c[1:, 1:] = a.cumsum(0).cumsum(1)
    K = 2 * r + 1
    return c[K:, K:] - c[:-K, K:] - c[K:, :-K] + c[:-K, :-K]


def fma32(a, b, c):
    """Correctly rounded float32 fma on arrays: a*b is exact in float64 and the
    one double rounding that can differ (the float64 sum landing exactly on a
    float32 midpoint) is resolved by the TwoSum error term."""
    a, b, c = (np.asarray(t, f32) for t in (a, b, c))
    p = a.astype(np.float64) * b.astype(np.float64)
    cd = c.astype(np.float64)
    s = p + cd
    bb = s - p
    err = (p - (s - bb)) + (cd - bb)
    r = s.astype(f32)
    rd = r.astype(np.float64)
    other = np.nextafter(r, np.where(s > rd, f32(np.inf), f32(-np.inf)).astype(f32))
    mid = (s != rd) & ((rd + other.astype(np.float64)) == 2 * s) & (err != 0)
    pick = np.where(err > 0, np.maximum(r, other), np.minimum(r, other))
    return np.where(mid, pick, r).astype(f32)


def _inv_sqrt_var(v):
    vf = np.where(v != 0, v, 1).astype(f32)
    return np.where(v != 0, f32(1) / np.sqrt(vf), f32(0)).astype(f32)


def ncc_volume(q, levels, vs, sn, aw, bl, K, z):
    """Build-defined NCC K x K cost volume (csrc/ncc.hip header) -> [D][H][W]:
    1 - max(-1, s_r * max over valid neighbour windows of
    fma(-Sr', Sp' s_p, Srp' (n s_p))), centred sums, s = 1/sqrt(var)."""
    V, H, W = q.shape
    r, nk = K // 2, K * K
    bl = f32(bl)
    qr = q[z].astype(np.int64) - 128
    rx, ry = z % aw, z // aw
    Sr = np.zeros((H, W), np.int64)
    Srr = np.zeros((H, W), np.int64)
    Sr[r:H - r, r:W - r] = _box(qr, r)
    Srr[r:H - r, r:W - r] = _box(qr * qr, r)
    sr = _inv_sqrt_var(nk * Srr - Sr * Sr)
    y, x = np.mgrid[0:H, 0:W]
    rin = (x - r >= 0) & (x + r < W) & (y - r >= 0) & (y + r < H)
    vol = np.zeros((len(levels), H, W), f32)
    for dl, d in enumerate(np.asarray(levels, f32)):
        best = np.full((H, W), -np.inf, f32)
        for n in range(sn[z]):
            view = vs[z, n]
            dx, dy = view % aw - rx, view // aw - ry
            tx = int(roundf(d * f32(dx)))
            ty = int(roundf((bl * d) * f32(dy)))
            qp = q[view].astype(np.int64) - 128
            Sp = np.zeros((H, W), np.int64)
            Spp = np.zeros((H, W), np.int64)
            Srp = np.zeros((H, W), np.int64)
            # shifted neighbour: p(y, x) = qp[y - ty, x - tx]
            sh = np.zeros((H, W), np.int64)
            ys0, ys1 = max(0, ty), min(H, H + ty)
            xs0, xs1 = max(0, tx), min(W, W + tx)
            if ys0 < ys1 and xs0 < xs1:
                sh[ys0:ys1, xs0:xs1] = qp[ys0 - ty:ys1 - ty, xs0 - tx:xs1 - tx]
            Sp[r:H - r, r:W - r] = _box(sh, r)
            Spp[r:H - r, r:W - r] = _box(sh * sh, r)
            Srp[r:H - r, r:W - r] = _box(qr * sh, r)
            px, py = x - tx, y - ty
            ok = rin & (px - r >= 0) & (px + r < W) & (py - r >= 0) & (py + r < H)
            sp = _inv_sqrt_var(nk * Spp - Sp * Sp)
            ap = (f32(nk) * sp).astype(f32)
            bp = (Sp.astype(f32) * sp).astype(f32)
            e = fma32(-Sr.astype(f32), bp, (Srp.astype(f32) * ap).astype(f32))
            best = np.where(ok & (e > best), e, best).astype(f32)
        with np.errstate(invalid="ignore"):
            E = (best * sr).astype(f32)  # -inf * 0 = NaN: no valid window
        vol[dl] = f32(1) - np.where(E > f32(-1), E, f32(-1)).astype(f32)
    return vol


def wta(vol, levels):
    """First argmin over [D][H][W]; conf = min outside best+-1 minus best."""
    D = vol.shape[0]
    bi = np.argmin(vol, 0)  # first minimum
    best = np.take_along_axis(vol, bi[None], 0)[0]
    d = np.arange(D)[:, None, None]
    masked = np.where(np.abs(d - bi[None]) <= 1, f32(1e6), vol)
    c2 = masked.min(0)
    conf = np.where(c2 == f32(1e6), f32(0), c2 - best).astype(f32)
    disp = np.asarray(levels, f32)[bi]
    # a pixel whose every cost is >= 1e6 keeps the default disparity 0
    none = best >= f32(1e6)
    return np.where(none, f32(0), disp), np.where(none, f32(0), conf)


def edge(lab):
    """edge_compute_alternative (clcode.cl:161-195): the magnitude of the
    reference's Sobel-like operator (DX uses the centre c4), clamped 3x3
    neighbourhood, float32 left to right; dot(v, 1) = (v.x + v.y) + v.z."""
    lab = np.asarray(lab, np.float32)
    H, W = lab.shape[:2]
    ys = np.clip(np.arange(H)[:, None] + np.array([-1, 0, 1])[None, :], 0, H - 1)
    xs = np.clip(np.arange(W)[:, None] + np.array([-1, 0, 1])[None, :], 0, W - 1)
    c = [lab[ys[:, yo + 1]][:, xs[:, xo + 1], :3] for yo in (-1, 0, 1) for xo in (-1, 0, 1)]
    f = np.float32
    dx = f(-1) * c[0] + c[2]
    dx = dx - f(2) * c[3]
    dx = dx + f(2) * c[4]
    dx = dx - c[5]
    dx = dx + c[7]
    dy = f(-1) * c[0] - f(2) * c[1]
    dy = dy - c[2]
    dy = dy + c[5]
    dy = dy + f(2) * c[6]
    dy = dy + c[7]
    s = dx * dx + dy * dy
    return np.sqrt((s[..., 0] + s[..., 1]) + s[..., 2]).astype(np.float32)


def apply_edge(lab, e, spixl):
    """apply_edge_alternative (clcode.cl:204-248) on one view's centres."""
    H, W = e.shape
    sp = np.array(spixl, np.float32, copy=True)
    dxy = [(-1, 0), (-1, -1), (0, -1), (1, -1), (1, 0), (1, 1), (0, 1), (-1, 1)]
    for s in sp.reshape(-1, 8):
        cx, cy = int(s[1]), int(s[2])
        if not (0 <= cx < W and 0 <= cy < H):
            continue
        ev, best = e[cy, cx], None
        for ox, oy in dxy:
            nx, ny = cx + ox, cy + oy
            if 0 <= nx < W and 0 <= ny < H and e[ny, nx] < ev:
                ev, best = e[ny, nx], (nx, ny)
        if best is not None:
            s[1], s[2] = best
            s[3:6] = lab[best[1], best[0], :3]
    return sp
