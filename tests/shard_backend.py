"""CPU stand-in for distributed.EngineBackend, computing each stage with the
oracle, so that the view-sharded orchestration (block split, in-place
gathers, per-iteration state exchange, filter gather) runs under gloo on CPU.
Test infrastructure only."""
from __future__ import annotations

import numpy as np
import torch

from oracle import oracle as orc


def _np(t):
    return t.detach().cpu().numpy()


def _lab(t):
    """Label maps as uint32: int32 bits, or 16-bit maps (the narrowed gather) widened."""
    a = _np(t)
    return a.view(np.uint32) if a.dtype.itemsize == 4 else a.view(np.uint16).astype(np.uint32)


class OracleBackend:
    def cvt(self, rgbx, views):
        # only the listed views are converted; the rest stay NaN / 0xff so a
        # stage reading a view outside its block's needs shows up as a mismatch
        x = _np(rgbx)
        lab = np.full(x.shape, np.nan, np.float32)
        q = np.full(x.shape[:3], 255, np.uint8)
        for v in views:
            lab[v] = orc.cvt(x[v])
            q[v] = orc.l8(lab[v])
        return torch.from_numpy(lab), torch.from_numpy(q)

    def slic(self, lab_blk, S, weight, no_iter, conn, search=0):
        lab = _np(lab_blk)
        outs = [orc.slic_from_lab(lab[v], S, weight, no_iter, conn, search) for v in range(lab.shape[0])]
        sp = np.stack([o[0] for o in outs]) if outs else np.zeros((0,), np.float32)
        lb = np.stack([o[1] for o in outs]).view(np.int32)
        return torch.from_numpy(sp), torch.from_numpy(lb)

    def boundary(self, spixl, labels, S, z0, z1):
        rep = np.full(tuple(spixl.shape[:3]) + (8,), 255, np.uint8)
        rep[z0:z1] = orc.boundary(_np(spixl)[z0:z1], _lab(labels)[z0:z1], S)
        return torch.from_numpy(rep)

    def sweep_spixl(self, lab, spixl, rep, cam, S, z0, z1):
        sp = orc.sweep(_np(lab), _np(spixl), _np(rep), cam.levels, cam.view_subset, cam.subset_num,
                       cam.array_width, cam.bl_ratio, S, z0, z1)
        spixl.copy_(torch.from_numpy(sp))

    def pixel_sweep(self, lab, l8, cam, z0, z1, cost, K, views):
        if cost == "sad":
            d = orc.sweep_pixel_sad(_np(lab), cam.levels, cam.view_subset, cam.subset_num, cam.array_width,
                                    cam.bl_ratio, z0, z1)
            return torch.from_numpy(d), None
        q = _np(l8)
        ds, cs = [], []
        for z in range(z0, z1):
            vol = orc.ncc_volume(q, cam.levels, cam.view_subset, cam.subset_num, cam.array_width, cam.bl_ratio, K, z)
            d, c = orc.wta(vol, cam.levels)
            ds.append(d)
            cs.append(c)
        return torch.from_numpy(np.stack(ds)), torch.from_numpy(np.stack(cs))

    def flatness(self, spixl, gamma):
        return torch.from_numpy(orc.flatness(_np(spixl), gamma))

    def init_state(self, spixl, labels, rep, flat, cam, S, gamma, alpha, nks, kss, fuse, z0, z1):
        r = np.zeros_like(_np(rep))  # the oracle runs every view: give the others harmless extents
        r[z0:z1] = _np(rep)[z0:z1]
        st = orc.init_state(_np(spixl), _lab(labels), r, _np(flat), cam.view_subset,
                            cam.subset_num, cam.array_width, cam.bl_ratio, S, gamma, alpha, nks, kss, fuse)
        out = np.full(st.shape, np.nan, np.float32)
        out[z0:z1] = st[z0:z1]
        return torch.from_numpy(out)

    def propagate(self, spixl, labels, rep, flat, cam, S, it, alpha, gamma, fuse, nks, kss, st_in, st_out, z0, z1):
        out = orc.propagate(_np(spixl), _lab(labels), _np(rep), _np(flat), cam.view_subset,
                            cam.subset_num, cam.array_width, cam.bl_ratio, S, it, alpha, gamma, fuse, nks, kss,
                            _np(st_in), z0, z1)
        st_out[z0:z1] = torch.from_numpy(out[z0:z1])
        return st_out

    def spixl_to_image(self, spixl, labels, state, S):
        return torch.from_numpy(orc.spixl_to_image(_np(spixl), _lab(labels), _np(state), S))

    def proj_inv(self, disp_full, aw, bl, z0, z1, proj=None, rows=None, band=False):
        oproj, _ = orc.filt(_np(disp_full), aw, bl, 1.0)
        out = torch.full(oproj.shape, float("nan")) if proj is None else proj
        ya, yb = rows if rows is not None else (0, oproj.shape[1])
        if band:  # proj is the row band alone, [V, yb - ya, W]
            out[z0:z1] = torch.from_numpy(oproj[z0:z1, ya:yb])
        else:
            out[z0:z1, ya:yb] = torch.from_numpy(oproj[z0:z1, ya:yb])
        return out

    def remove_inconsistency(self, disp_full, proj, aw, bl, fuse, z0, z1, out=None, rows=None, band=False):
        # the oracle filter recomputes every projection itself: check that the
        # gathered proj rows the product orchestration hands over equal it
        oproj, filt = orc.filt(_np(disp_full), aw, bl, fuse)
        ya, yb = rows if rows is not None else (0, oproj.shape[1])
        got = _np(proj) if band else _np(proj)[:, ya:yb]
        if not np.array_equal(got.view(np.uint32), oproj[:, ya:yb].view(np.uint32)):
            raise AssertionError("gathered proj slices differ from the full projection")
        res = torch.zeros_like(disp_full) if out is None else out
        res[z0:z1, ya:yb] = torch.from_numpy(filt[z0:z1, ya:yb])
        return res
