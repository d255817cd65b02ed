"""The view-sharded pipeline (cl_multiview_stereo_amd/distributed.py) under
gloo on CPU, world_size 1/2/3: a sharded run must give bit-identical depth
maps to the unsharded single-process computation, for equal and ragged view
blocks.  Compute comes from the oracle stand-in (tests/shard_backend.py); the
orchestration and the collectives are the product code."""
from __future__ import annotations

import os
import socket
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _case(name):
    from tests.cases import CASES, build
    c = dict(CASES[name])
    return c, build(c)


def _settings(c):
    from cl_multiview_stereo_amd import params
    return params.Settings(spixl_size=c["S"], array_width=c["aw"], array_height=c["ah"], neib_hor=c["nh"],
                           neib_ver=c["nv"], min_disp=c["dmin"], max_disp=c["dmax"], bl_ratio=c["bl"],
                           kernel_size=52, no_prop=3, window=5)


def _unsharded(c, b):
    from oracle import oracle as orc
    S = c["S"]
    outs = [orc.slic(b["stack"][v], S) for v in range(b["V"])]
    lab = np.stack([o[0] for o in outs])
    sp = np.stack([o[1] for o in outs])
    lb = np.stack([o[2] for o in outs])
    rep = orc.boundary(sp, lb, S)
    sp = orc.sweep(lab, sp, rep, b["levels"], b["vs"], b["sn"], c["aw"], c["bl"], S)
    ref = orc.refine(sp, lb, rep, b["vs"], b["sn"], c["aw"], c["bl"], S, kernel_size=52, no_prop=3)
    _, filt = orc.filt(ref["disp"], c["aw"], c["bl"], 1.0)
    q = orc.l8(lab)
    disp = np.stack([orc.wta(orc.ncc_volume(q, b["levels"], b["vs"], b["sn"], c["aw"], c["bl"], 5, z),
                             b["levels"])[0] for z in range(b["V"])])
    return dict(spixl=sp, labels=lb, refined=ref["disp"], filt=filt, disp=disp)


def _worker(rank, world, port, name, outdir, bands=None, shard=None):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from cl_multiview_stereo_amd.distributed import ShardedPipeline, ViewGather
    from cl_multiview_stereo_amd.engine import CameraArray
    from shard_backend import OracleBackend
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c, b = _case(name)
        st = _settings(c)
        cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], b["sn"])
        g = ViewGather(b["V"])
        pipe = ShardedPipeline(OracleBackend(), st, cam, g, pixel_cost="ncc", refine=True, filt=True, proj_bands=bands,
                               filter_shard=shard)
        out = pipe.run(torch.from_numpy(b["stack"]))
        np.savez(os.path.join(outdir, f"r{rank}.npz"), z=np.array([out.z0, out.z1]), spixl=out.spixl.numpy(),
                 labels=out.labels32().numpy().view(np.uint32), disp=out.disp.numpy(),
                 refined=out.disp_refined.numpy(), filt=out.disp_filtered.numpy())
    finally:
        dist.destroy_process_group()


# shard: the filter's sharding ("rows", the default, or "views"); bands: row
# bands of the "views" form's pipelined proj all-gather (None: 2 at world > 1)
@pytest.mark.parametrize("name,world,bands,shard", [("c3x1_s8", 2, None, "rows"), ("c3x1_s8", 3, None, "rows"),
                                                    ("c2x2_s12", 2, None, "rows"), ("c2x2_s12", 3, None, "rows"),
                                                    ("c3x1_s8", 2, None, "views"),
                                                    ("c3x1_s8", 3, None, "views"), ("c2x2_s12", 2, 1, "views"),
                                                    ("c3x1_s8", 1, None, "rows"), ("c3x1_s8", 1, 3, "views")])
def test_sharded_equals_unsharded(name, world, bands, shard):
    c, b = _case(name)
    want = _unsharded(c, b)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(world, _free_port(), name, d, bands, shard), nprocs=world, join=True,
                           start_method="spawn")
        seen = []
        for r in range(world):
            with np.load(os.path.join(d, f"r{r}.npz")) as z:
                z0, z1 = (int(v) for v in z["z"])
                seen.append((z0, z1))
                assert np.array_equal(z["labels"], want["labels"])
                assert np.array_equal(z["spixl"].view(np.uint32), want["spixl"].view(np.uint32))
                for k in ("disp", "refined", "filt"):
                    assert np.array_equal(z[k].view(np.uint32), want[k][z0:z1].view(np.uint32)), (r, k)
        # the blocks tile [0, V) exactly
        assert seen[0][0] == 0 and seen[-1][1] == b["V"]
        assert all(seen[i][1] == seen[i + 1][0] for i in range(world - 1))


def test_view_block_partition():
    from cl_multiview_stereo_amd.distributed import all_blocks, view_block
    for V in range(1, 40):
        for world in range(1, 9):
            blocks = all_blocks(V, world)
            sizes = [z1 - z0 for z0, z1 in blocks]
            assert sum(sizes) == V and max(sizes) - min(sizes) <= 1
            assert blocks[0][0] == 0 and blocks[-1][1] == V
    assert all_blocks(32, 8) == [(4 * r, 4 * r + 4) for r in range(8)]  # C4: 4 views per GPU
    with pytest.raises(ValueError):
        view_block(4, 4, 4)


def test_gather_single_process_is_copy():
    from cl_multiview_stereo_amd.distributed import ViewGather
    g = ViewGather(3)
    x = torch.arange(12.0).reshape(3, 4)
    assert torch.equal(g(x), x)
    with pytest.raises(ValueError):
        g(x[:2])


def _gather_worker(rank, world, port, outdir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from cl_multiview_stereo_amd.distributed import ViewGather
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = ViewGather(4 * world)
        z0, z1 = g.block
        full = torch.full((4 * world, 5), -1.0)
        full[z0:z1] = torch.arange(20.0).reshape(4, 5) + 100 * rank
        pend = g.start(full[z0:z1], full)  # async, in place (all_gather_into_tensor, async_op=True)
        got = pend.wait()
        assert got.data_ptr() == full.data_ptr() and pend.wait() is full
        np.save(os.path.join(outdir, f"g{rank}.npy"), got.numpy())
    finally:
        dist.destroy_process_group()


def test_async_gather_gloo():
    """ViewGather.start (the labels all-gather the sharded pipeline overlaps
    with its sweeps) equals the blocks of every rank, world 2."""
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_gather_worker, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
        want = np.concatenate([np.arange(20.0).reshape(4, 5) + 100 * r for r in range(2)]).astype(np.float32)
        for r in range(2):
            assert np.array_equal(np.load(os.path.join(d, f"g{r}.npy")), want)


def test_labels_16bit_round_trip():
    """The 16-bit labels gather (distributed._narrow_labels): int32 -> int16
    (wrap) -> bytes -> int16 -> uint16 -> int32 is the identity on 0..65535."""
    from cl_multiview_stereo_amd.distributed import _bytes
    t = torch.arange(0, 1 << 16, dtype=torch.int32).view(4, 128, 128)
    l16 = t.to(torch.int16)
    b = _bytes(l16).clone()
    back = b.view(torch.int16).view(4, 128, 128).view(torch.uint16).to(torch.int32)
    assert torch.equal(back, t)
