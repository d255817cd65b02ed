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


class OracleBackend:
    def cvt(self, rgbx):
        lab = orc.cvt(_np(rgbx))
        return torch.from_numpy(lab), torch.from_numpy(orc.l8(lab))

    def slic(self, lab_blk, S, weight, no_iter, conn):
        lab = _np(lab_blk)
        outs = [orc.slic_from_lab(lab[v], S, weight, no_iter, conn) for v in range(lab.shape[0])]
        sp = np.stack([o[0] for o in outs]) if outs else np.zeros((0,), np.float32)
        lb = np.stack([o[1] for o in outs]).view(np.int32)
        return torch.from_numpy(sp), torch.from_numpy(lb)

    def boundary(self, spixl, labels, S):
        return torch.from_numpy(orc.boundary(_np(spixl), _np(labels).view(np.uint32), S))

    def sweep_spixl(self, lab, spixl, rep, cam, S, z0, z1):
        sp = orc.sweep(_np(lab), _np(spixl), _np(rep), cam.levels, cam.view_subset, cam.subset_num,
                       cam.array_width, cam.bl_ratio, S, z0, z1)
        spixl.copy_(torch.from_numpy(sp))

    def pixel_sweep(self, lab, l8, cam, z0, z1, cost, K):
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

    def init_state(self, spixl, labels, rep, flat, cam, S, gamma, alpha, nks, kss, fuse):
        return torch.from_numpy(orc.init_state(_np(spixl), _np(labels).view(np.uint32), _np(rep), _np(flat),
                                               cam.view_subset, cam.subset_num, cam.array_width, cam.bl_ratio, S,
                                               gamma, alpha, nks, kss, fuse))

    def propagate(self, spixl, labels, rep, flat, cam, S, it, alpha, gamma, fuse, nks, kss, st_in, st_out, z0, z1):
        out = orc.propagate(_np(spixl), _np(labels).view(np.uint32), _np(rep), _np(flat), cam.view_subset,
                            cam.subset_num, cam.array_width, cam.bl_ratio, S, it, alpha, gamma, fuse, nks, kss,
                            _np(st_in), z0, z1)
        st_out[z0:z1] = torch.from_numpy(out[z0:z1])
        return st_out

    def spixl_to_image(self, spixl, labels, state, S):
        return torch.from_numpy(orc.spixl_to_image(_np(spixl), _np(labels).view(np.uint32), _np(state), S))

    def filter(self, disp_full, aw, bl, fuse, z0, z1):
        _, out = orc.filt(_np(disp_full), aw, bl, fuse)
        res = torch.zeros_like(disp_full)
        res[z0:z1] = torch.from_numpy(out[z0:z1])
        return res
