"""The view-sharded pipeline over RCCL (torch.distributed "nccl" on ROCm):
world 2, one process per GPU, the HIP engine on each rank's device.  The
sharded run must give the unsharded oracle's depth maps bit for bit -- the
same bar as tests/test_distributed_cpu.py (gloo + oracle stand-in), here with
the product compute and the overlapped collectives on real streams: the async
in-place labels all-gather (16-bit) still in flight during the sweeps, and the
row-sharded cross-view filter's point-to-point rows -> views exchange (and the
reference-view form's row-banded proj all-gather).

Skipped with fewer than 2 GPUs visible (the round's 1-GPU boxes); the
driver's multi-GPU node runs it."""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tests.test_distributed_cpu import ROOT, _case, _free_port, _settings, _unsharded

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs 2 GPUs (RCCL world 2)")]


def _worker(rank, world, port, name, outdir, bands, shard):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    from cl_multiview_stereo_amd.distributed import EngineBackend, ShardedPipeline, ViewGather
    from cl_multiview_stereo_amd.engine import CameraArray, Engine
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    try:
        c, b = _case(name)
        e = Engine(rank)
        cam = CameraArray(c["aw"], c["bl"], b["levels"], b["vs"], b["sn"])
        pipe = ShardedPipeline(EngineBackend(e, fused=True), _settings(c), cam, ViewGather(b["V"]), pixel_cost="ncc",
                               refine=True, filt=True, proj_bands=bands, filter_shard=shard)
        out = pipe.run(torch.from_numpy(b["stack"]).cuda())
        torch.cuda.synchronize()
        np.savez(os.path.join(outdir, f"r{rank}.npz"), z=np.array([out.z0, out.z1]), spixl=out.spixl.cpu().numpy(),
                 labels=out.labels32().cpu().numpy().view(np.uint32), disp=out.disp.cpu().numpy(),
                 refined=out.disp_refined.cpu().numpy(), filt=out.disp_filtered.cpu().numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("name,bands,shard", [("c3x1_s8", None, "rows"), ("c2x2_s12", None, "views"),
                                              ("c2x2_s12", 1, "views")])
def test_sharded_rccl_equals_unsharded(name, bands, shard):
    c, b = _case(name)
    want = _unsharded(c, b)
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_worker, args=(2, _free_port(), name, d, bands, shard), nprocs=2, join=True,
                           start_method="spawn")
        for r in range(2):
            with np.load(os.path.join(d, f"r{r}.npz")) as z:
                z0, z1 = (int(v) for v in z["z"])
                assert np.array_equal(z["labels"], want["labels"])
                assert np.array_equal(z["spixl"].view(np.uint32), want["spixl"].view(np.uint32))
                for k in ("disp", "refined", "filt"):
                    assert np.array_equal(z[k].view(np.uint32), want[k][z0:z1].view(np.uint32)), (r, k)


def _gather_worker(rank, world, port, outdir):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    import torch.distributed as dist
    from cl_multiview_stereo_amd.distributed import ViewGather
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", rank))
    try:
        g = ViewGather(4 * world)
        z0, z1 = g.block
        full = torch.full((4 * world, 5), -1.0, device="cuda")
        full[z0:z1] = torch.arange(20.0, device="cuda").reshape(4, 5) + 100 * rank
        got = g.start(full[z0:z1], full).wait()
        np.save(os.path.join(outdir, f"g{rank}.npy"), got.cpu().numpy())
    finally:
        dist.destroy_process_group()


def test_async_gather_rccl():
    with tempfile.TemporaryDirectory() as d:
        mp.start_processes(_gather_worker, args=(2, _free_port(), d), nprocs=2, join=True, start_method="spawn")
        want = np.concatenate([np.arange(20.0).reshape(4, 5) + 100 * r for r in range(2)]).astype(np.float32)
        for r in range(2):
            assert np.array_equal(np.load(os.path.join(d, f"g{r}.npy")), want)
