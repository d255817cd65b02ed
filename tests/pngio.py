"""Tiny PNG reader/writer for the tests (zlib only): writes every 8-bit colour
type with any of the five scanline filters, so the C++ loader of mvs_cli is
exercised on all of them, and reads what mvs_cli writes."""
from __future__ import annotations

import struct
import zlib

import numpy as np

CH = {0: 1, 2: 3, 4: 2, 6: 4}


def _chunk(t: bytes, d: bytes) -> bytes:
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xffffffff)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return np.where((pa <= pb) & (pa <= pc), a, np.where(pb <= pc, b, c))


def write_png(path: str, px: np.ndarray, ctype: int, filt: int | str = 0) -> None:
    """px: [H][W][ch] uint8.  filt: 0..4, or 'mixed' (row y uses filter y % 5)."""
    H, W = px.shape[:2]
    ch = CH[ctype]
    img = px.reshape(H, W * ch).astype(np.int32)
    rows = []
    for y in range(H):
        f = (y % 5) if filt == "mixed" else int(filt)
        cur = img[y]
        up = img[y - 1] if y else np.zeros_like(cur)
        left = np.concatenate([np.zeros(ch, np.int32), cur[:-ch]])
        ul = np.concatenate([np.zeros(ch, np.int32), up[:-ch]])
        pred = [np.zeros_like(cur), left, up, (left + up) // 2, _paeth(left, up, ul)][f]
        rows.append(bytes([f]) + ((cur - pred) % 256).astype(np.uint8).tobytes())
    raw = b"".join(rows)
    data = (b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 8, ctype, 0, 0, 0)) +
            _chunk(b"IDAT", zlib.compress(raw, 6)) + _chunk(b"IEND", b""))
    with open(path, "wb") as f:
        f.write(data)


def read_png_gray(path: str) -> np.ndarray:
    b = open(path, "rb").read()
    assert b[:8] == b"\x89PNG\r\n\x1a\n"
    p, idat, W, H = 8, b"", 0, 0
    while p < len(b):
        n = struct.unpack(">I", b[p:p + 4])[0]
        t, d = b[p + 4:p + 8], b[p + 8:p + 8 + n]
        if t == b"IHDR":
            W, H, depth, ctype = struct.unpack(">IIBB", d[:10])
            assert depth == 8 and ctype == 0
        elif t == b"IDAT":
            idat += d
        p += 12 + n
    raw = zlib.decompress(idat)
    out = np.zeros((H, W), np.uint8)
    for y in range(H):
        assert raw[y * (W + 1)] == 0  # mvs_cli writes filter 0
        out[y] = np.frombuffer(raw[y * (W + 1) + 1:(y + 1) * (W + 1)], np.uint8)
    return out
