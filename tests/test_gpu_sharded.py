"""GPU: the view-sharded pipeline on the HIP backend (world 1) equals the
unsharded oracle, and every view-ranged entry point ([z0, z1) arguments of
mvs_sweep_spixl_d / mvs_propagate_d / mvs_filter_d) computes exactly its
block, so per-rank blocks tile the unsharded result."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from cl_multiview_stereo_amd import params
from cl_multiview_stereo_amd.distributed import EngineBackend, ShardedPipeline, ViewGather, all_blocks
from cl_multiview_stereo_amd.engine import CameraArray
from tests.cases import CASES, build
from tests.test_distributed_cpu import _settings, _unsharded

pytestmark = pytest.mark.gpu


def bits(a):
    a = a.cpu().numpy() if hasattr(a, "cpu") else np.asarray(a)
    return a.view(np.uint32) if a.dtype in (np.float32, np.int32) else a


@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("name", ["c3x1_s8", "c2x2_s12"])
def test_sharded_pipeline_world1(engine, name, fused):
    c = dict(CASES[name])
    b = build(c)
    want = _unsharded(c, b)
    cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], b["sn"])
    pipe = ShardedPipeline(EngineBackend(engine, fused=fused), _settings(c), cam, ViewGather(b["V"]))
    out = pipe.run(torch.from_numpy(b["stack"]).cuda())
    assert np.array_equal(bits(out.labels), want["labels"])
    assert np.array_equal(bits(out.spixl), want["spixl"].view(np.uint32))
    for k, t in (("disp", out.disp), ("refined", out.disp_refined), ("filt", out.disp_filtered)):
        assert np.array_equal(bits(t), want[k].view(np.uint32)), k


@pytest.mark.parametrize("world", [2, 3])
def test_view_ranges_tile_the_full_result(engine, world):
    c = dict(CASES["c3x3_s8"])
    b = build(c)
    V, S = b["V"], c["S"]
    lab, _ = engine.cvt(torch.from_numpy(b["stack"]).cuda())
    sp, lb = engine.slic(lab, S)
    rep = engine.boundary(sp, lb, S)
    cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], b["sn"])
    full = sp.clone()
    engine.sweep_spixl(lab, full, rep, cam, S)
    part = sp.clone()
    for z0, z1 in all_blocks(V, world):
        engine.sweep_spixl(lab, part, rep, cam, S, z0, z1)
    assert torch.equal(full, part)
    rp = params.refine_params(params.Settings(spixl_size=S, kernel_size=52))
    flat = engine.flatness(full, rp["flat_gamma"])
    st = engine.init_state(full, lb, rep, flat, cam, S, rp["init_gamma"], rp["init_alpha"], rp["kernel_steps"],
                           rp["kss"], rp["fuse"])
    nks, kss = params.prop_schedule(0, rp["kernel_steps"], rp["kss"])
    a = torch.zeros_like(st)
    engine.propagate(full, lb, rep, flat, cam, S, 0, rp["prop_alpha"], rp["prop_gamma"], rp["fuse"], nks, kss, st, a)
    bpart = torch.zeros_like(st)
    for z0, z1 in all_blocks(V, world):
        engine.propagate(full, lb, rep, flat, cam, S, 0, rp["prop_alpha"], rp["prop_gamma"], rp["fuse"], nks, kss,
                         st, bpart, z0, z1)
    assert torch.equal(a, bpart)
    disp = engine.spixl_to_image(full, lb, a, S)
    _, f_full = engine.filter(disp, c["aw"], c["bl"], 1.0)
    f_part = torch.zeros_like(f_full)
    for z0, z1 in all_blocks(V, world):
        _, o = engine.filter(disp, c["aw"], c["bl"], 1.0, z0, z1)
        f_part[z0:z1] = o[z0:z1]
    assert torch.equal(f_full, f_part)
