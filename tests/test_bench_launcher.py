"""bench.py's multi-GPU launch path on CPU (gloo, --dry-run): `--gpus N`
without WORLD_SIZE spawns N ranks itself, a torch.distributed.run launch
takes them from the environment, and either way rank 0 prints ONE JSON line
with n_gpus == N after a ViewGather over all ranks."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _json_lines(out):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("n", [1, 2, 3])
def test_spawn_launcher(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus", str(n), "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == n and lines[0]["world_size"] == n and lines[0]["gather_ok"]
    assert lines[0]["steps"] == 2 and lines[0]["warmup"] == 1


def test_torchrun_launch():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
                        "--dry-run", "--gpus", "2", "--steps", "2", "--warmup", "1"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2 and lines[0]["gather_ok"]


def test_world_size_mismatch_is_refused():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--gpus", "2"],
                       capture_output=True, text=True, timeout=120, env=env, cwd=ROOT)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


_GUARD = """
import sys, time
sys.path.insert(0, {root!r})
import bench
def vs(*a):
    if {mode!r} == "raise":
        raise RuntimeError("collective failed")
    time.sleep(60)
bench.view_sharded = vs
r = bench._guarded_view_sharded(None, None, 2, 0, None, {{"metric": "m", "value": 1.0}})
print("returned", r, flush=True)
bench._WATCH["done"].set()
"""


@pytest.mark.parametrize("mode", ["raise", "hang"])
def test_sharded_subline_guard(mode):
    """The C4 sub-line at world > 1 cannot take the headline line with it: an
    exception comes back as {"error": ...}; a hang trips the watchdog, which
    prints the line without the field and ends the rank with status 3 (a hung
    collective must fail the run, never pass as rc 0)."""
    env = _env()
    env["MVS_SHARDED_TIMEOUT"] = "2"
    p = subprocess.run([sys.executable, "-c", _GUARD.format(root=ROOT, mode=mode)], env=env, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == (0 if mode == "raise" else 3), p.stderr
    if mode == "raise":
        assert "returned {'error': \"RuntimeError('collective failed')\"}" in p.stdout
    else:
        (line,) = _json_lines(p.stdout)
        assert line["value"] == 1.0 and "error" in line["view_sharded"]
        assert "returned" not in p.stdout


_HANG = """
import os, sys, time
sys.path.insert(0, {root!r})
import torch, torch.distributed as dist
import bench
from cl_multiview_stereo_amd.distributed import ViewGather
dist.init_process_group("gloo")
rank = dist.get_rank()

def vs(args, e, world, rank, sync):
    # the sharded leg's own all-gather; rank 1 never joins it, so rank 0's
    # collective hangs inside gloo exactly as a stuck RCCL gather would
    g = ViewGather(4)
    full = torch.zeros((4, 8))
    z0, z1 = g.block
    if rank == 1:
        time.sleep(120)
    g(full[z0:z1], full)
    return {{"ok": True}}

bench.view_sharded = vs
r = bench._guarded_view_sharded(None, None, 2, rank, None, {{"metric": "m", "value": 1.0}})
print("returned", r, flush=True)
"""


def test_hung_collective_fails_the_run(tmp_path):
    """A gloo world-2 job whose sharded leg hangs in a real all-gather (rank 1
    never joins): the watchdog prints the headline line on rank 0 with the
    sharded field set to an error, and the job exits non-zero."""
    script = tmp_path / "hang.py"
    script.write_text(_HANG.format(root=ROOT))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = _env()
    env["MVS_SHARDED_TIMEOUT"] = "3"
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)],
                       capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode != 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert line["value"] == 1.0 and "error" in line["view_sharded"]
    assert "returned" not in r.stdout


@pytest.mark.parametrize("config", ["c2", "c5"])
def test_committed_pmc_feeds_roofline_headline(config):
    """The driver line's roofline_headline comes from the committed PMC summary
    of the fused sweep (profiles/pmc_ncc_<config>.json, scripts/summarize_prof.py):
    it must carry the per-view VALU count for the bench shape, and its source
    must exist in the tree."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    cfg = bench.CONFIGS[config]
    got = bench._valu_insts_fused_per_view(config, cfg["W"], cfg["H"], cfg["dmax"] - cfg["dmin"] + 1)
    assert got is not None and got["insts"] > 0
    assert os.path.exists(os.path.join(root, got["source"]))
