"""C4's whole workload against the oracle: the 8 x 4 camera array, every view a
reference with its 5 nearest neighbours (params.nearest_neighbours), through
the view-sharded pipeline on the HIP backend -- SLIC, extents, superpixel
sweep, fused NCC 5x5 sweep + WTA over 128 levels, refinement (5 propagations,
compute_consistency over the 5-NN lists, clcode.cl:1528-1631) and the
cross-view filter -- on a 256 x 128 crop with S = 16 and on a 384 x 192 crop
with C4's own S = 32 (the tile-fused SLIC path, k_assign_tiles +
k_update_finalize, that the full-size C4 run takes).

* world 1: the product orchestration (ViewGather) on one GPU;
* world 8: each rank r of a world of 8 runs ShardedPipeline with a replay of
  the world-1 gathers (tests/replay_gather.py): it computes only its block of
  4 views and reads the other views exactly as an RCCL all-gather would
  deliver them.

Labels, centres + seeds, NCC disparity, refined and filtered depth of every
view must equal the unsharded oracle's bit for bit."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from cl_multiview_stereo_amd import params, synth
from cl_multiview_stereo_amd.distributed import EngineBackend, ShardedPipeline, ViewGather
from cl_multiview_stereo_amd.engine import CameraArray
from oracle import oracle as orc
from tests.replay_gather import RecordingGather, ReplayGather

AW, AH, DMAX = 8, 4, 127
GEOMS = {"s16": (256, 128, 16), "s32": (384, 192, 32)}  # crop W, H and superpixel size S


def _case(geom="s16"):
    W, H, S = GEOMS[geom]
    # a scene 0..15 px deep, swept over 128 hypotheses (C4's 0..127 levels)
    stack, _ = synth.make_stack(W, H, AW, AH, 0, 15, 1.0, 0xC4)
    levels = params.disparity_levels(0, DMAX, 1)
    vs, sn = params.flatten_subsets(params.nearest_neighbours(AW, AH, 5))
    st = params.Settings(spixl_size=S, array_width=AW, array_height=AH, min_disp=0, max_disp=DMAX, inc=1,
                         bl_ratio=1.0, window=5, cost="ncc")
    return stack, levels, vs, sn, st


_ORACLE = {}


def _oracle(geom="s16"):
    if geom in _ORACLE:
        return _ORACLE[geom]
    stack, levels, vs, sn, st = _case(geom)
    S = st.spixl_size
    V = AW * AH
    outs = [orc.slic(stack[v], S) for v in range(V)]
    lab = np.stack([o[0] for o in outs])
    sp = np.stack([o[1] for o in outs])
    lb = np.stack([o[2] for o in outs])
    rep = orc.boundary(sp, lb, S)
    sp = orc.sweep(lab, sp, rep, levels, vs, sn, AW, 1.0, S)
    q = orc.l8(lab)
    disp = np.stack([orc.wta(orc.ncc_volume(q, levels, vs, sn, AW, 1.0, 5, z), levels)[0] for z in range(V)])
    ref = orc.refine(sp, lb, rep, vs, sn, AW, 1.0, S)  # main()'s refinement settings
    _, filt = orc.filt(ref["disp"], AW, 1.0, 1.0)
    _ORACLE[geom] = dict(labels=lb, spixl=sp, disp=disp, refined=ref["disp"], filt=filt)
    return _ORACLE[geom]


def _bits(t):
    a = t.cpu().numpy() if hasattr(t, "cpu") else np.asarray(t)
    return a.view(np.uint32)


def _check(out, want, z0, z1):
    """Gathered labels / spixl of every view, and the rank's own block of maps."""
    assert np.array_equal(_bits(out.labels32()), want["labels"]), "labels"
    assert np.array_equal(_bits(out.spixl), want["spixl"].view(np.uint32)), "spixl (centres + seeds)"
    for k, t in (("disp", out.disp), ("refined", out.disp_refined), ("filt", out.disp_filtered)):
        assert np.array_equal(_bits(t), want[k][z0:z1].view(np.uint32)), k


@pytest.mark.gpu
@pytest.mark.parametrize("geom", sorted(GEOMS))
def test_c4_world1_matches_oracle(engine, geom):
    stack, levels, vs, sn, st = _case(geom)
    want = _oracle(geom)
    cam = CameraArray(AW, 1.0, levels, vs, sn)
    pipe = ShardedPipeline(EngineBackend(engine, fused=True), st, cam, ViewGather(AW * AH), pixel_cost="ncc",
                           refine=True, filt=True)
    out = pipe.run(torch.from_numpy(stack).cuda())
    _check(out, want, 0, AW * AH)


@pytest.mark.gpu
@pytest.mark.parametrize("shard,geom", [("rows", "s16"), ("views", "s16"), ("rows", "s32")])
def test_c4_world8_replay_matches_oracle(engine, shard, geom):
    """shard: the filter sharded by image rows (the default: every reference
    view's rows of the rank's band, then the rows -> views exchange) or by
    reference view (row-banded proj all-gather)."""
    stack, levels, vs, sn, st = _case(geom)
    want = _oracle(geom)
    V = AW * AH
    cam = CameraArray(AW, 1.0, levels, vs, sn)
    be = EngineBackend(engine, fused=True)
    rgbx = torch.from_numpy(stack).cuda()
    rg = RecordingGather(V)
    kw = dict(pixel_cost="ncc", refine=True, filt=True, proj_bands=2, filter_shard=shard)
    ShardedPipeline(be, st, cam, rg, **kw).run(rgbx)
    for r in range(8):
        g = ReplayGather(V, r, 8, list(rg.rec))
        out = ShardedPipeline(be, st, cam, g, **kw).run(rgbx)
        z0, z1 = g.block
        assert (z0, z1) == (4 * r, 4 * r + 4)
        _check(out, want, z0, z1)
