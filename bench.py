#!/usr/bin/env python3
"""Headline benchmark: Mpix/s of per-view depth on synthetic 5-view 1080p
stacks, 128 disparity hypotheses, NCC 5x5, SLIC K~2000 (BASELINE.json config 2).

One step = the whole depth pipeline over one batch: for each of the V reference
views of this rank's stack (inputs RGBx already resident in HBM): Lab
conversion, SLIC (S=32, 5 update/assign iterations), superpixel extents, the
reference superpixel SAD sweep, the per-pixel NCC 5x5 sweep over 128
hypotheses x 4 neighbours and its winner-take-all + confidence.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--cost ncc|sad]

`value` is the fused step (mvs_ncc_wta_d: the sweep kernel folds the WTA in,
no cost volume in HBM), on one HIP stream (--concurrent: the superpixel chain
on a side stream; `concurrent_variant` times that form too).  The same invocation also times the two-pass step
(materialised [D][H][W] volume + the k_wta streaming pass, bit-identical maps):
`roofline` is k_wta's HBM read of that volume, the north star's roofline.

N>1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) the
ranks come from the environment; `--gpus N` without WORLD_SIZE spawns the N
rank processes itself before anything touches a GPU.  Every rank owns its own
5-view stack (independent objects, no data-path collective) -> weak scaling;
`view_sharded` adds C4 (one 32-view array sharded by reference view over the
N GPUs, RCCL all-gathers, the filter sharded by rows with a point-to-point
rows -> views exchange) -> strong scaling.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

CONFIGS = {
    # name: (array w, h, W, H, S, dmin, dmax, K, nh, nv, bl)
    "c1": dict(aw=2, ah=1, W=640, H=480, S=1, dmin=0, dmax=31, K=5, nh=1, nv=0, bl=1.0, cost="sad",
               workload="2-view 640x480, 32 hypotheses, SAD 5x5, SLIC off (reference per-pixel sweep)"),
    "c2": dict(aw=5, ah=1, W=1920, H=1080, S=32, dmin=0, dmax=127, K=5, nh=4, nv=0, bl=1.0, cost="ncc",
               workload="5-view 1920x1080, 128 hypotheses, NCC 5x5, SLIC K=2040 (S=32), 1 GPU per 5-view stack"),
    "c3": dict(aw=5, ah=1, W=1920, H=1080, S=32, dmin=0, dmax=127, K=5, nh=4, nv=0, bl=1.0, cost="ncc",
               refine=True, filt=True,
               workload="C2 + superpixel refinement (5 propagations) + cross-view consistency filter, 1 GPU per stack"),
    "c4": dict(aw=8, ah=4, W=1920, H=1080, S=32, dmin=0, dmax=127, K=5, nh=0, nv=0, knn=5, bl=1.0, cost="ncc",
               refine=True, filt=True, sharded=True,
               workload="32 reference views x 5 nearest neighbours, 1080p, one array sharded by reference view over "
                        "the GPUs (RCCL all-gathers of labels/spixl and refinement state, fused maps rendered per "
                        "rank, projections gathered in row bands)"),
    # the reference's own defaults (clMVDE.cpp main): its algorithm exactly, no per-pixel sweep
    "ref": dict(aw=3, ah=3, W=1920, H=1080, S=8, dmin=30, dmax=60, K=5, nh=1, nv=1, bl=1.0359, cost="none",
                refine=True,
                workload="clMVDE main() defaults: 3x3 array 1080p, S=8 (32,400 superpixels/view), levels 30..60, "
                         "superpixel SAD sweep + refinement (5 propagations) + fusion, all 9 views"),
    "c5": dict(aw=5, ah=1, W=4096, H=3072, S=40, dmin=0, dmax=255, K=7, nh=4, nv=0, bl=1.0, cost="ncc",
               workload="5-view 4096x3072, 256 hypotheses, NCC 7x7, SLIC K=7931 (S=40)"),
}
METRIC = "Mpix/s depth (1080p, 128 depth hyp, 5 views) + depth L1 vs ref"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
VALU_PEAK = 1024 * 2.4e9 / 4.0  # wave64 VALU instructions/s: 1024 SIMDs x 2.4 GHz / 4 cycles
VALU_PEAK_NOTE = ("1024 SIMDs x 2.4 GHz / 4 cycles per wave64 instruction: profiles/r05/valu_rate3.txt measures "
                  "v_dot4_i32_i8 / v_pk_fma_f32 / v_pk_mul_f32 / v_max_f32 / v_med3_f32 at 4.13-4.35 cycles per "
                  "wave-instruction per SIMD at 4-8 waves per SIMD (v_add_f32 / v_mul_f32 / v_mov_b32 2.2-2.5, "
                  "v_fma_f32 3.6-3.8); the sweep's mix weighs in at ~3.9")
CPU_SAMPLE_SECONDS = 15.0  # target CPU time of the per-pixel sweep's sampled row band (cpu_baseline)
CPU_TAP_RATE = {"ncc": 13e9, "sad": 8e9}  # oracle taps/s on the GPU box's 16 host threads (measured r02)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cost", default=None, choices=["ncc", "sad", "none"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sharded", action="store_true", help="skip the C4 view-sharded strong-scaling line")
    ap.add_argument("--no-reference-cost", action="store_true", help="skip the C2 --cost sad sub-line")
    ap.add_argument("--no-reference-defaults", action="store_true",
                    help="skip the `reference_defaults` sub-line (--config ref inside the c2 line)")
    ap.add_argument("--no-c3", action="store_true",
                    help="skip the `c3` sub-line (--config c3: refinement + consistency filter, inside the c2 line)")
    ap.add_argument("--two-pass", action="store_true",
                    help="headline = the two-pass step (cost volume in HBM + k_wta) instead of the fused sweep")
    ap.add_argument("--concurrent", action="store_true",
                    help="superpixel chain on a second stream beside the per-pixel chain (pipeline.py); one "
                         "stream is the default (`concurrent_variant` times this form beside the headline)")
    # a no-op since round 5 (one stream is the default): accepted so that the
    # command lines of the round-3/4 records still run
    ap.add_argument("--serial", action="store_true", help="no-op: one stream is the default (old command lines)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the launcher, rank setup, gathers and max-over-ranks timing on gloo")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher: one process per GPU
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_entry(rank, args, port):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    run(args)


def main(argv=None):
    args = parse(argv)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # spawn the ranks before anything initialises a GPU in this process
        import torch.multiprocessing as mp
        mp.start_processes(_rank_entry, args=(args, _free_port()), nprocs=args.gpus, join=True, start_method="spawn")
        return
    run(args)


def _ranks():
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def _max_over_ranks(x, device, world):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed(step, steps, warmup, device, world, sync):
    """W untimed warmup steps, then EXACTLY K steps between barrier + sync on
    both sides; the max over ranks of the elapsed time, and the last output."""
    import torch.distributed as dist
    out = None
    for _ in range(warmup):
        out = step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    sync()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    return _max_over_ranks(t1 - t0, device, world), out


def run(args):
    world, rank, local = _ranks()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    if args.dry_run:
        return dry_run(args, world, rank)
    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        assert dist.get_world_size() == world
    try:
        res = bench(args, world, rank, local)
        if rank == 0:
            _emit(res)
    finally:
        if world > 1:
            dist.destroy_process_group()
        _WATCH["done"].set()


_WATCH = {"done": threading.Event(), "printed": False, "lock": threading.Lock()}
WATCHDOG_EXIT = 3  # a hung sharded collective: the line is printed, the run still fails


def _emit(res):
    """Print the one JSON line (once: the sharded watchdog may print it first)."""
    with _WATCH["lock"]:
        if not _WATCH["printed"]:
            _WATCH["printed"] = True
            print(json.dumps(res), flush=True)


def _guarded_view_sharded(args, e, world, rank, sync, res):
    """The C4 sub-line, never at the cost of the headline line: an exception is
    reported in the field, and at world > 1 -- where the sharded collectives
    (async all-gathers, the point-to-point row exchange) run over RCCL -- a
    watchdog armed until the process is done prints the line without the field
    and ends the rank after MVS_SHARDED_TIMEOUT seconds (default 180) if they
    hang: the headline is still reported, but the rank exits with status 3, so
    a hung collective fails the run instead of passing as rc 0."""
    if world > 1:
        limit = float(os.environ.get("MVS_SHARDED_TIMEOUT", "180"))

        def watch():
            if _WATCH["done"].wait(limit):
                return
            if rank == 0:
                out = dict(res)
                out["view_sharded"] = {"error": f"no result within {limit:.0f} s; rank exited by the bench watchdog"}
                _emit(out)
            log(f"rank {rank}: sharded sub-line watchdog fired after {limit:.0f} s; exiting with status 3")
            sys.stdout.flush()
            os._exit(WATCHDOG_EXIT)

        threading.Thread(target=watch, daemon=True).start()
    try:
        return view_sharded(args, e, world, rank, sync)
    except Exception as ex:  # report, never hide; the headline stands
        return {"error": repr(ex)}


def dry_run(args, world, rank):
    """The launch/timing/reporting path without a GPU: gloo ranks, one
    ViewGather (the product's all-gather) of a 5-view block per step."""
    import torch
    import torch.distributed as dist

    from cl_multiview_stereo_amd.distributed import ViewGather
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == world
    g = ViewGather(5 * world)
    full = torch.zeros((5 * world, 64, 64))
    z0, z1 = g.block

    def step():
        full[z0:z1] = float(rank + 1)
        return g(full[z0:z1], full)

    el, out = timed(step, args.steps, args.warmup, "cpu", world, lambda: None)
    ok = all(bool((out[b0:b1] == r + 1).all()) for r, (b0, b1) in enumerate(g.blocks))
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "Mpix/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(el * 1e3 / max(args.steps, 1), 4),
                          "dry_run": True, "gather_ok": ok, "world_size": world}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def _cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = None
    quota = None
    try:  # cgroup v2 CPU quota: "max 100000" or "<quota> <period>"
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = {"cpu.max": f"{q} {per}", "cpus": None if q == "max" else round(int(q) / int(per), 2)}
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "nproc": os.cpu_count(), "affinity_cpus": affinity,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS"), "cgroup_cpu_quota": quota}


def _pmc_traffic(name, W, H, D):
    """Corrected HBM bytes per launch of k_wta from this configuration's own
    PMC pass (profiles/pmc_wta_<config>.json, written by scripts/profile.sh),
    or None when no pass of this exact shape exists."""
    p = os.path.join(ROOT, "profiles", f"pmc_wta_{name}.json")
    if not os.path.exists(p):
        return None
    try:
        j = json.load(open(p))
    except (OSError, ValueError):
        return None
    if (j.get("W"), j.get("H"), j.get("D")) != (W, H, D):
        return None
    return j.get("hbm_bytes_per_launch")


def _valu_insts(name, cost, fused, W, H, D):
    """SQ_INSTS_VALU per launch of the (plain, one view per launch) NCC sweep
    from this configuration's own PMC pass (profiles/pmc_ncc_<config>.json,
    scripts/profile.sh), launch-weighted over the band-width variants; None
    without a pass of this shape."""
    pmc_ncc = os.path.join(ROOT, "profiles", f"pmc_ncc_{name}.json")
    if cost != "ncc" or not os.path.exists(pmc_ncc):
        return None
    j = json.load(open(pmc_ncc))
    if (j.get("W"), j.get("H"), j.get("D")) != (W, H, D):
        return None
    tag = "true>" if fused else "false>"
    ent = [v for k, v in j.items() if k.startswith("k_ncc_volume") and k.endswith(tag)]
    if not ent:
        return None
    wts = [e.get("launches", 1) for e in ent]
    return sum(e["valu_wave_insts_per_launch"] * w for e, w in zip(ent, wts)) / sum(wts)


def _valu_insts_fused_per_view(name, W, H, D):
    """SQ_INSTS_VALU of the fused sweep per reference view: the PMC pass's
    total over every fused launch divided by the reference views its bench
    process swept (profile_counts.ncc_wta_views of that run's own JSON line,
    recorded by scripts/summarize_prof.py as fused_valu_wave_insts_per_view).
    "stale" is set when the NCC sources changed since that pass (the summary
    records their hash), so no fraction is quoted on another kernel's counts."""
    p = os.path.join(ROOT, "profiles", f"pmc_ncc_{name}.json")
    if not os.path.exists(p):
        return None
    j = json.load(open(p))
    if (j.get("W"), j.get("H"), j.get("D")) != (W, H, D) or "fused_valu_wave_insts_per_view" not in j:
        return None
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from summarize_prof import ncc_src_sha16
    now = ncc_src_sha16(ROOT)
    kern = next((k for k in j if k.startswith("k_ncc_mfma")), None) or next(
        (k for k in j if k.startswith("k_ncc_volume") and ", true" in k), "k_ncc_volume<..., FUSE=true>")
    out = {"insts": j["fused_valu_wave_insts_per_view"], "source": j.get("source"),
           "mfma": j.get("fused_mfma_insts_per_view", 0.0), "kernel": kern}
    if j.get("ncc_src_sha16") != now:
        out["stale"] = (f"the PMC pass ({j.get('source')}) counted NCC sources {j.get('ncc_src_sha16')}, this tree "
                        f"is {now}: no fraction quoted until scripts/profile.sh is re-run")
    return out


def bench(args, world, rank, local):
    import torch

    from cl_multiview_stereo_amd import params, synth
    from cl_multiview_stereo_amd.engine import Engine
    from cl_multiview_stereo_amd.pipeline import Pipeline

    cfg = dict(CONFIGS[args.config])
    cost = args.cost or cfg["cost"]
    V = cfg["aw"] * cfg["ah"]
    W, H = cfg["W"], cfg["H"]
    D = cfg["dmax"] - cfg["dmin"] + 1
    st = params.Settings(spixl_size=cfg["S"], array_width=cfg["aw"], array_height=cfg["ah"], min_disp=cfg["dmin"],
                         max_disp=cfg["dmax"], inc=1, neib_hor=cfg["nh"], neib_ver=cfg["nv"], bl_ratio=cfg["bl"],
                         window=cfg["K"], cost=cost)
    e = Engine(local)
    dev = e.device
    sync = torch.cuda.synchronize
    sharded = bool(cfg.get("sharded"))
    fused = cost == "ncc" and not args.two_pass
    # independent stacks per rank (weak scaling) or one array sharded by view (strong)
    stack, _ = synth.make_stack(W, H, cfg["aw"], cfg["ah"], cfg["dmin"], cfg["dmax"], cfg["bl"],
                                0x5EED + 2 + (0 if sharded else rank))
    rgbx = torch.from_numpy(stack).to(dev)
    vlists = params.nearest_neighbours(cfg["aw"], cfg["ah"], cfg["knn"]) if cfg.get("knn") else None

    # HIP events around the sweep / WTA launches, on the stream they run on
    # (engine calls are enqueued on torch's current stream: Engine._stream).
    # Every call is counted, timed or not, so a PMC pass of this same command
    # can divide its counter totals by calls (scripts/summarize_prof.py).
    timers = {"wta": [], "ncc": [], "fused": []}
    calls = {"wta": 0, "ncc": 0, "fused": 0, "fused_views": 0}
    recording = [False]

    def instrument(name, fn, views=None):
        def w(*a, **k):
            s = torch.cuda.Event(enable_timing=True)
            t = torch.cuda.Event(enable_timing=True)
            s.record()
            r = fn(*a, **k)
            t.record()
            n = views(*a, **k) if views else 1
            calls[name] += 1
            if name == "fused":
                calls["fused_views"] += n
            if recording[0]:
                timers[name].append((s, t, n))
            return r
        return w

    e.wta = instrument("wta", e.wta)
    e.ncc_volume = instrument("ncc", e.ncc_volume)
    e.ncc_wta = instrument("fused", e.ncc_wta)
    # the fused path of Pipeline: one call per run of reference views [z0, z1)
    e.ncc_wta_range = instrument("fused", e.ncc_wta_range, views=lambda l8, box, cam, z0, z1, *a, **k: z1 - z0)

    def avg(lst):
        return sum(s.elapsed_time(t) for s, t, _ in lst) / len(lst) * 1e-3

    # One HIP stream for the whole step (the default since round 5).  The
    # superpixel chain on a side stream beside the per-pixel chain
    # (pipeline.py, concurrent=True; --concurrent) bought 0.05 % in round 4
    # and 0.2 % with the matrix-core sweep (2.0673 vs 2.0716 ms per C2 step,
    # profiles/r05/bench_default_conc.json): both chains are throughput-bound,
    # so sharing the CUs only moves time between them.  Its A/B stays in the
    # line as `concurrent_variant`.
    conc_head = bool(args.concurrent) or os.environ.get("MVS_BENCH_CONCURRENT") == "1"  # (env: interleaved A/B)

    def make(fz, conc=False):
        p = Pipeline(e, st, W, H, view_subset=vlists, pixel_cost=None if cost == "none" else cost,
                     refine=bool(cfg.get("refine")), filt=bool(cfg.get("filt")) and not sharded,
                     concurrent=conc, fused=fz)
        if not sharded:
            return p, (lambda: p.exe_pipeline(rgbx))
        from cl_multiview_stereo_amd.distributed import EngineBackend, ShardedPipeline, ViewGather
        sp = ShardedPipeline(EngineBackend(e, fused=fz), st, p.cam, ViewGather(V), pixel_cost=cost, refine=True,
                             filt=bool(cfg.get("filt")))
        return p, (lambda: sp.run(rgbx))

    pipe, step = make(fused, conc_head)
    recording[0] = True
    # the fused sweep's own dispatch time as well (events of its launches,
    # hipExtLaunchKernel): an event recorded on the stream before a call can
    # fire while the previous kernel still runs (the ring sweep, ~0.16 ms), so
    # the call-bracketing events read ~5 % high (profiles/r05/headline_check.json)
    ktimes, kviews = None, 0
    views0 = calls["fused_views"]
    if fused and hasattr(e, "set_kernel_timing"):
        e.set_kernel_timing(True)
    elapsed, out = timed(step, args.steps, args.warmup, dev, world, sync)
    recording[0] = False
    if fused and hasattr(e, "set_kernel_timing"):
        ktimes = e.kernel_times()
        kviews = calls["fused_views"] - views0  # the views those launches swept (warmup + timed steps)
        e.set_kernel_timing(False)
    ms_per_step = elapsed * 1e3 / max(args.steps, 1)
    units = V if sharded else world * V  # reference views processed per step, whole job
    mpix = units * W * H * args.steps / elapsed / 1e6
    head_timers = {k: list(v) for k, v in timers.items()}
    form_timers = head_timers  # the headline's own form (side stream included): roofline_headline
    serial = None
    if conc_head:
        # the same step on one stream: the fused kernel's own time for
        # roofline_sweep (beside the side stream it shares the CUs)
        _, ser_step = make(fused, False)
        for k in timers:
            timers[k].clear()
        recording[0] = True
        ser_el, ser_out = timed(ser_step, args.steps, max(1, args.warmup), dev, world, sync)
        recording[0] = False
        head_timers = {k: list(v) for k, v in timers.items()}
        serial = {"what": "the same step on one HIP stream (the headline runs the superpixel chain on a side "
                          "stream beside the per-pixel chain)",
                  "value": round(units * W * H * args.steps / ser_el / 1e6, 3), "unit": "Mpix/s",
                  "ms_per_step": round(ser_el * 1e3 / max(args.steps, 1), 4),
                  "bit_identical_to_headline": bool(all(
                      torch.equal(getattr(ser_out, f).view(torch.int32), getattr(out, f).view(torch.int32))
                      for f in ("disp", "conf") if getattr(out, f, None) is not None))}

    conc_var = None
    if not conc_head and fused and not sharded and cost == "ncc" and world == 1:
        _, conc_step = make(fused, True)
        saved = {k: list(v) for k, v in timers.items()}
        c_el, c_out = timed(conc_step, args.steps, max(1, args.warmup), dev, world, sync)
        for k in timers:  # the headline's own timers stay the ones of the headline pass
            timers[k][:] = saved[k]
        conc_var = {"what": "the same step with the superpixel chain on a side HIP stream beside the per-pixel "
                            "chain (--concurrent)",
                    "value": round(units * W * H * args.steps / c_el / 1e6, 3), "unit": "Mpix/s",
                    "ms_per_step": round(c_el * 1e3 / max(args.steps, 1), 4),
                    "bit_identical_to_headline": bool(all(
                        torch.equal(getattr(c_out, f).view(torch.int32), getattr(out, f).view(torch.int32))
                        for f in ("disp", "conf") if getattr(out, f, None) is not None))}

    res = {
        "metric": METRIC,
        "value": round(mpix, 3),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if sharded else "weak",
        "vs_baseline": None,
        "dtype": ("i8 (NCC: 8-bit intensities as int8 v_dot4 operands, i32 window sums, f32 costs; "
                  "SLIC / superpixel SAD / refinement in f32 with the reference's f64 promotions)") if cost == "ncc"
                 else "f32 (Lab SAD, the reference's arithmetic; f64 where its double literals promote)",
        "data": "synthetic (seeded rendered camera-array stack, RGBx resident in HBM)",
        "config": {"name": args.config, "workload": cfg["workload"] if cost == cfg["cost"] else
                   cfg["workload"].replace("NCC", f"{cost.upper()} (--cost {cost}) instead of NCC"), "views": V, "width": W, "height": H, "hypotheses": D,
                   "window": cfg["K"], "cost": cost, "spixl_size": cfg["S"],
                   "neighbours": int(pipe.cam.subset_num.max()),
                   "sweep": ("fused sweep + WTA (no cost volume in HBM)" if fused else
                             "two-pass (cost volume in HBM + k_wta)") if cost == "ncc" else cost,
                   "parallelism": (f"views sharded over {world} GPU(s)" if sharded else
                                   f"view-stack per GPU x{world}"),
                   "refinement": bool(cfg.get("refine")), "consistency_filter": bool(cfg.get("filt")),
                   "streams": "superpixel chain on a side stream" if conc_head else "one"},
    }
    if serial is not None:
        res["serial_variant"] = serial
    if conc_var is not None:
        res["concurrent_variant"] = conc_var
    if fused and head_timers["fused"]:
        t_f = avg(head_timers["fused"])  # per call (one run of reference views)
        vpc = sum(n for _, _, n in head_timers["fused"]) / len(head_timers["fused"])
        cells = float(D) * W * H
        nbr = max(1, int(pipe.cam.subset_num[0]))
        per_view = _valu_insts_fused_per_view(args.config, W, H, D)
        res["roofline_sweep"] = {
            "kernel": "fused sweep + WTA (k_ncc_mfma: K = 5 lists, K = 7 horizontal lists; k_ncc_volume<..., FUSE=true> where its bands miss the LDS): the headline step's dominant kernel",
            "bound": "valu", "avg_call_ms": round(t_f * 1e3, 4), "views_per_call": vpc,
            "avg_ms_per_view": round(t_f * 1e3 / vpc, 4),
            "view_cells_per_s": round(cells * nbr * vpc / t_f / 1e9, 3), "unit_view_cells": "G view-cells/s",
            "timing": "HIP events around each mvs_ncc_wta_range_d call of the timed steps, on its stream" +
                      (" (the serial_variant pass: one stream, the kernel alone on the GPU)" if conc_head else "")}
        if ktimes and kviews > 0 and not conc_head:
            res["roofline_sweep"]["kernel_avg_ms_per_view"] = round(sum(ktimes) / kviews, 4)
            res["roofline_sweep"]["kernel_timing"] = ("start / stop events of each fused launch's own dispatch "
                                                      "(hipExtLaunchKernel), warmup + timed steps")
        if per_view is not None and not per_view.get("stale"):
            valu_only = per_view["insts"] - per_view.get("mfma", 0.0)  # (SQ_INSTS_VALU counts the MFMAs)
            res["roofline_sweep"].update({
                "valu_wave_insts_per_view": round(valu_only),
                "valu_issue_frac": round(valu_only * vpc / t_f / VALU_PEAK, 4),
                "valu_peak": VALU_PEAK_NOTE,
                "valu_source": per_view["source"]})
        if per_view is not None:
            # the roofline of the kernel the headline step spends its time in,
            # timed in the headline's own form (side stream beside it) and, for
            # reference, alone on one stream (the serial pass)
            def form(tm):
                tf = avg(tm["fused"])
                vp = sum(n for _, _, n in tm["fused"]) / len(tm["fused"])
                return tf, vp
            t_h, v_h = form(form_timers) if form_timers["fused"] else (t_f, vpc)
            t_ev = t_h
            # the kernel's own dispatch time per call when recorded (warmup + timed
            # calls alike: every recorded call's views over every recorded launch)
            kview = None
            if ktimes and form_timers["fused"] and not conc_head and kviews > 0:
                kview = sum(ktimes) * 1e-3 / kviews
                t_h = kview * v_h
            # SQ_INSTS_VALU counts the MFMAs too: the vector ALU's
            # own instructions are the difference; the matrix core is a separate
            # pipe, reported on its own line (busy share at 16 cycles per
            # v_mfma_i32_16x16x64_i8, the cycles of the bf16 16x16x32 form)
            mf = per_view.get("mfma", 0.0)
            valu = per_view["insts"] - mf
            ach = valu * v_h / t_h / 1e9
            rh = {"bound": "valu", "kernel": per_view["kernel"],
                  "achieved": round(ach, 1), "peak": round(VALU_PEAK / 1e9, 1), "unit": "G VALU wave-instr/s",
                  "frac": round(ach * 1e9 / VALU_PEAK, 4),
                  "frac_guide_2cyc": round(ach * 1e9 / (2.0 * VALU_PEAK), 4),
                  "form": "headline (superpixel chain on the side stream)" if conc_head else "headline (one stream)",
                  "algorithmic": f"{round(valu)} vector-ALU wave-instructions per reference view (SQ_INSTS_VALU "
                                 f"{round(per_view['insts'])} minus SQ_INSTS_MFMA {round(mf)}, its own PMC pass, "
                                 f"{per_view['source']}) over the "
                                 + ("kernel's own dispatch time per view (start / stop events of its launches, "
                                    "hipExtLaunchKernel)" if kview is not None else "HIP-event time per view")
                                 + " in the headline pass",
                  "avg_ms_per_view": round(t_h * 1e3 / v_h, 4),
                  "event_avg_ms_per_view": round(t_ev * 1e3 / v_h, 4),
                  "peak_basis": VALU_PEAK_NOTE + "; frac_guide_2cyc: the same at MI355X_MICROARCH.md's 2 cycles per "
                                                 "wave64 instruction (1,228.8 G/s)"}
            if mf:
                rh["mfma"] = {"insts_per_view": round(mf),
                              "pipe_busy_frac": round(mf * 16.0 * v_h / t_h / (1024 * 2.4e9), 4),
                              "basis": "16 matrix-core cycles per v_mfma_i32_16x16x64_i8 on its SIMD, 1024 SIMDs x "
                                       "2.4 GHz"}
            if conc_head:
                rh["serial_form"] = {"avg_ms_per_view": round(t_f * 1e3 / vpc, 4),
                                     "frac": round(valu * vpc / t_f / VALU_PEAK, 4)}
            if per_view.get("stale"):
                rh.update({"frac": None, "frac_guide_2cyc": None, "achieved": None, "stale_pmc": per_view["stale"]})
            res["roofline_headline"] = rh

    # the two-pass step (cost volume in HBM + k_wta), same protocol: the
    # north star's roofline is k_wta's read of that volume
    if cost == "ncc":
        tp_out = out
        if fused:
            _, tp_step = make(False, False)
            for k in timers:
                timers[k].clear()
            recording[0] = True
            tp_el, tp_out = timed(tp_step, args.steps, max(1, args.warmup), dev, world, sync)
            recording[0] = False
            same = all(torch.equal(getattr(tp_out, f).view(torch.int32), getattr(out, f).view(torch.int32))
                       for f in ("disp", "conf") if getattr(out, f, None) is not None)
            res["two_pass_variant"] = {"what": "the same step with the cost volume materialised in HBM + k_wta",
                                       "value": round(units * W * H * args.steps / tp_el / 1e6, 3), "unit": "Mpix/s",
                                       "ms_per_step": round(tp_el * 1e3 / max(args.steps, 1), 4),
                                       "bit_identical_to_headline": bool(same)}
        if timers["wta"]:
            t_wta = avg(timers["wta"])
            t_ncc = avg(timers["ncc"])
            wta_bytes = 4.0 * D * W * H + 8.0 * W * H  # volume read + disparity/confidence write
            achieved = wta_bytes / t_wta / 1e9
            res["roofline"] = {"bound": "hbm",
                               "kernel": "k_wta (cost-volume read pass of the two-pass step, timed in this run)",
                               "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(achieved / HBM_PEAK_GBS, 4),
                               "traffic": _pmc_traffic(args.config, W, H, D),
                               "algorithmic_bytes_per_launch": wta_bytes, "avg_launch_ms": round(t_wta * 1e3, 4)}
            cells = float(D) * W * H
            nbr = max(1, int(pipe.cam.subset_num[0]))
            sw = {"kernel": "k_ncc_volume (cost-volume write pass)", "avg_launch_ms": round(t_ncc * 1e3, 4),
                  "view_cells_per_s": round(cells * nbr / t_ncc / 1e9, 3), "unit_view_cells": "G view-cells/s",
                  "hbm_write_GBps": round(4.0 * cells / t_ncc / 1e9, 1),
                  "hbm_write_frac": round(4.0 * cells / t_ncc / 1e9 / HBM_PEAK_GBS, 4)}
            insts = _valu_insts(args.config, cost, False, W, H, D)
            if insts is not None:
                sw.update({"bound": "valu", "valu_wave_insts_per_launch": round(insts),
                           "valu_issue_frac": round(insts / t_ncc / VALU_PEAK, 4)})
            res.setdefault("two_pass_variant", {})["roofline_sweep"] = sw

    # PCIe-inclusive rate: the RGBx stack H2D from pinned host memory and the
    # disparity maps D2H inside the timed region (never `value`)
    if not sharded and world == 1 and hasattr(out, "disp"):
        host_in = torch.from_numpy(stack).pin_memory()
        src = out.disp_refined if out.disp is None else out.disp
        host_out = torch.empty(tuple(src.shape), dtype=torch.float32).pin_memory()
        dev_in = torch.empty_like(rgbx)

        def pstep():
            dev_in.copy_(host_in, non_blocking=True)
            o = pipe.exe_pipeline(dev_in)  # the headline pipeline
            host_out.copy_(o.disp_refined if o.disp is None else o.disp, non_blocking=True)
            return o

        p_el, _ = timed(pstep, args.steps, 1, dev, world, sync)
        res["pcie_inclusive"] = {"value": round(V * W * H * args.steps / p_el / 1e6, 3), "unit": "Mpix/s",
                                 "ms_per_step": round(p_el * 1e3 / max(args.steps, 1), 4),
                                 "what": f"H2D of the {stack.nbytes / 1e6:.1f} MB RGBx stack (pinned) + the step "
                                         f"+ D2H of the {host_out.numel() * 4 / 1e6:.1f} MB disparity maps"}

    # the reference's own arithmetic (SAD over Lab, clcode.cl:1030-1053) on the
    # headline shape: the only cost against which the north star's L1 target
    # is defined (C2 with --cost sad, 3 steps)
    if args.config == "c2" and cost == "ncc" and world == 1 and not args.no_reference_cost:
        res["reference_cost"] = reference_cost(args, e, st, stack, rgbx, cfg, world, sync,
                                               check=rank == 0 and not args.no_cpu_baseline)

    # the reference's own algorithm at its own defaults (clMVDE.cpp:14-36), so a
    # regression of its kernels (k_propagate above all) shows in the driver's line
    if args.config == "c2" and cost == "ncc" and world == 1 and not args.no_reference_defaults:
        try:
            res["reference_defaults"] = reference_defaults(args, e, world, sync,
                                                           check=rank == 0 and not args.no_cpu_baseline)
        except Exception as ex:  # report, never hide; the headline stands
            res["reference_defaults"] = {"error": repr(ex)}

    # BASELINE config 3 (C2 + refinement + consistency filter) inside the default
    # line, its refined and filtered maps against the oracle's full-size run
    if args.config == "c2" and cost == "ncc" and world == 1 and not args.no_c3:
        try:
            res["c3"] = c3_subline(args, e, world, sync, check=rank == 0 and not args.no_cpu_baseline)
        except Exception as ex:  # report, never hide; the headline stands
            res["c3"] = {"error": repr(ex)}

    # C4: one 32-view array sharded by reference view over the N GPUs (strong scaling)
    if not args.no_sharded and args.config in ("c2",) and cost == "ncc":
        res["view_sharded"] = _guarded_view_sharded(args, e, world, rank, sync, res)

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            if sharded:
                res["cpu_baseline"], res["depth_l1_vs_oracle"] = cpu_baseline_sharded_crop(e, cfg)
            else:
                res["cpu_baseline"], res["depth_l1_vs_oracle"] = cpu_baseline(pipe, stack, cfg, cost, out)
        except Exception as ex:  # report, never hide
            res["cpu_baseline"] = {"error": repr(ex)}
    # every sweep call this process made (warmup, timed, two-pass, PCIe and C4
    # legs): a PMC pass of this same command divides its totals by these
    res["profile_counts"] = {"ncc_wta_calls": calls["fused"], "ncc_wta_views": calls["fused_views"],
                             "ncc_volume_calls": calls["ncc"], "wta_calls": calls["wta"]}
    return res


def reference_cost(args, e, st, stack, rgbx, cfg, world, sync, check=True):
    """C2 with the reference's SAD cost (initial_depth_estimation_v2 at S = 1,
    the per-pixel k_sad_band sweep) instead of the build-defined NCC: 3 timed
    steps after 1 warmup, and the depth L1 against the oracle on three 62-row
    bands of every reference view -- top, middle, bottom -- each computed from
    its rows plus the window's 2-row margin (with horizontal-only neighbours
    those rows equal the full image's: a few seconds of CPU)."""
    import dataclasses

    import torch

    from cl_multiview_stereo_amd.pipeline import Pipeline
    W, H = cfg["W"], cfg["H"]
    V = stack.shape[0]
    sst = dataclasses.replace(st, cost="sad")
    p = Pipeline(e, sst, W, H, pixel_cost="sad", refine=False, filt=False, fused=False)
    steps = 3
    el, out = timed(lambda: p.exe_pipeline(rgbx), steps, 1, e.device, world, sync)
    r = {"what": "the C2 step with the reference's cost (SAD over Lab, 5x5 sparse window, min over neighbours, "
                 "WTA; clcode.cl:972-1069 at S = 1) in place of NCC 5x5",
         "value": round(V * W * H * steps / el / 1e6, 3), "unit": "Mpix/s", "ms_per_step": round(el * 1e3 / steps, 4),
         "steps": steps, "dtype": "f32"}
    if check:
        from oracle import oracle as orc
        cam = p.cam
        keep, R = 62, 2  # rows per band; the 5x5 window's reach
        t0 = time.perf_counter()
        disp = out.disp.cpu().numpy()
        got, want, names = [], [], []
        for y0 in (0, H // 2 - keep // 2, H - keep):  # top, middle tile rows, bottom
            b0, b1 = max(0, y0 - R), min(H, y0 + keep + R)
            lab_band = orc.cvt(np.ascontiguousarray(stack[:, b0:b1]))
            w = orc.sweep_pixel_sad(lab_band, cam.levels, cam.view_subset, cam.subset_num, cfg["aw"], cfg["bl"])
            want.append(w[:, y0 - b0:y0 - b0 + keep])
            got.append(disp[:, y0:y0 + keep])
            names.append(f"{y0}..{y0 + keep - 1}")
        got, want = np.concatenate(got, 1), np.concatenate(want, 1)
        r["depth_l1_vs_oracle"] = {"value": float(np.abs(got - want).mean()),
                                   "bit_exact": bool(np.array_equal(got, want)),
                                   "bands": names,
                                   "sample": f"rows {', '.join(names)} (three {keep}-row bands, each from its own "
                                             f"rows + the window's {R}-row margin) of all {V} reference views, {W} "
                                             f"wide (oracle: {time.perf_counter() - t0:.1f} s on the host)"}
    return r


def reference_defaults(args, e, world, sync, check=True):
    """`--config ref` inside the default line: clMVDE main()'s defaults (3x3
    array 1080p, S = 8, levels 30..60, bl 1.0359, superpixel SAD sweep +
    refinement with 5 propagations + fusion of all 9 views).  5 timed steps
    after 1 warmup; with `check`, the fused maps of the last step against the
    oracle's full-size run (~5 s on the host)."""
    import torch

    from cl_multiview_stereo_amd import params, synth
    from cl_multiview_stereo_amd.pipeline import Pipeline
    c = CONFIGS["ref"]
    V, W, H = c["aw"] * c["ah"], c["W"], c["H"]
    st = params.Settings(spixl_size=c["S"], array_width=c["aw"], array_height=c["ah"], min_disp=c["dmin"],
                         max_disp=c["dmax"], inc=1, neib_hor=c["nh"], neib_ver=c["nv"], bl_ratio=c["bl"],
                         window=c["K"], cost="none")
    stack, _ = synth.make_stack(W, H, c["aw"], c["ah"], c["dmin"], c["dmax"], c["bl"], 0x5EED + 2)  # = --config ref
    rgbx = torch.from_numpy(stack).to(e.device)
    p = Pipeline(e, st, W, H, pixel_cost=None, refine=True, filt=False, fused=False)
    steps = 5
    el, out = timed(lambda: p.exe_pipeline(rgbx), steps, 1, e.device, world, sync)
    r = {"what": c["workload"], "value": round(V * W * H * steps / el / 1e6, 3), "unit": "Mpix/s",
         "ms_per_step": round(el * 1e3 / steps, 4), "steps": steps, "dtype": "f32 (f64 where the reference promotes)"}
    if check:
        cpu, l1 = cpu_baseline(p, stack, c, "none", out)
        r["depth_l1_vs_oracle"] = l1
        r["cpu_baseline"] = {k: cpu[k] for k in ("value", "unit", "cores", "kind", "sample")}
    return r


def c3_subline(args, e, world, sync, check=True):
    """`--config c3` inside the default line: the C2 step + superpixel
    refinement (5 propagations, fusion) + the cross-view consistency filter
    (project_to_reference_inv + remove_view_inconsistency, clcode.cl:1995-2101),
    5 views 1920x1080, with the headline's stream layout (superpixel chain on
    the side stream).  5 timed steps after 1 warmup; with `check`, the last
    step's refined and filtered maps (and labels, seeds) against the oracle's
    full-size run (segmentation, superpixel sweep, refinement, filter: ~3 s on
    the host; the per-pixel NCC maps are the headline's, checked there)."""
    import torch

    from cl_multiview_stereo_amd import params, synth
    from cl_multiview_stereo_amd.pipeline import Pipeline
    c = CONFIGS["c3"]
    V, W, H, S = c["aw"] * c["ah"], c["W"], c["H"], c["S"]
    st = params.Settings(spixl_size=S, array_width=c["aw"], array_height=c["ah"], min_disp=c["dmin"],
                         max_disp=c["dmax"], inc=1, neib_hor=c["nh"], neib_ver=c["nv"], bl_ratio=c["bl"],
                         window=c["K"], cost="ncc")
    stack, _ = synth.make_stack(W, H, c["aw"], c["ah"], c["dmin"], c["dmax"], c["bl"], 0x5EED + 2)  # = --config c3
    rgbx = torch.from_numpy(stack).to(e.device)
    p = Pipeline(e, st, W, H, pixel_cost="ncc", refine=True, filt=True, concurrent=bool(args.concurrent), fused=True)
    steps = 5
    el, out = timed(lambda: p.exe_pipeline(rgbx), steps, 1, e.device, world, sync)
    r = {"what": c["workload"], "value": round(V * W * H * steps / el / 1e6, 3), "unit": "Mpix/s",
         "ms_per_step": round(el * 1e3 / steps, 4), "steps": steps,
         "streams": "superpixel chain on a side stream" if args.concurrent else "one"}
    if check:
        from oracle import oracle as orc
        t0 = time.perf_counter()
        cam = p.cam
        outs = [orc.slic(stack[v], S) for v in range(V)]
        lab = np.stack([o[0] for o in outs])
        sp = np.stack([o[1] for o in outs])
        lb = np.stack([o[2] for o in outs])
        rep = orc.boundary(sp, lb, S)
        sp = orc.sweep(lab, sp, rep, cam.levels, cam.view_subset, cam.subset_num, c["aw"], c["bl"], S)
        ref = orc.refine(sp, lb, rep, cam.view_subset, cam.subset_num, c["aw"], c["bl"], S)["disp"]
        filt = orc.filt(ref, c["aw"], c["bl"], 1.0)[1]
        t_orc = time.perf_counter() - t0
        torch.cuda.synchronize()
        maps = {"labels": (out.labels.cpu().numpy().view(np.uint32), lb), "spixl": (out.spixl.cpu().numpy(), sp),
                "disp_refined": (out.disp_refined.cpu().numpy(), ref),
                "disp_filtered": (out.disp_filtered.cpu().numpy(), filt)}
        l1 = {}
        for k, (g, w) in maps.items():
            l1[k] = {"bit_exact": bool(np.array_equal(g, w))}
            if k.startswith("disp"):
                l1[k]["value"] = float(np.abs(g - w).mean())
        r["depth_l1_vs_oracle"] = {"value": l1["disp_filtered"]["value"], "unit": "px (mean |d_gpu - d_oracle|)",
                                   "bit_exact": all(v["bit_exact"] for v in l1.values()), "map": "disp_filtered",
                                   "maps": l1,
                                   "sample": f"the last timed step, all {V} views {W}x{H} (oracle: {t_orc:.1f} s on "
                                             f"the host)"}
    return r


def view_sharded(args, e, world, rank, sync):
    """C4 at this world size: 32 reference views x 5 nearest neighbours, 1080p,
    each rank owning a contiguous block of views (distributed.py)."""
    import torch

    from cl_multiview_stereo_amd import params, synth
    from cl_multiview_stereo_amd.distributed import EngineBackend, ShardedPipeline, ViewGather
    from cl_multiview_stereo_amd.engine import CameraArray
    c = CONFIGS["c4"]
    V, W, H = c["aw"] * c["ah"], c["W"], c["H"]
    st = params.Settings(spixl_size=c["S"], array_width=c["aw"], array_height=c["ah"], min_disp=c["dmin"],
                         max_disp=c["dmax"], inc=1, bl_ratio=c["bl"], window=c["K"], cost="ncc")
    stack, _ = synth.make_stack(W, H, c["aw"], c["ah"], c["dmin"], c["dmax"], c["bl"], 0x5EED + 2)  # = --config c4
    rgbx = torch.from_numpy(stack).to(e.device)
    mat, num = params.flatten_subsets(params.nearest_neighbours(c["aw"], c["ah"], c["knn"]))
    cam = CameraArray(c["aw"], c["bl"], params.disparity_levels(c["dmin"], c["dmax"], 1), mat, num)
    g = ViewGather(V)
    sp = ShardedPipeline(EngineBackend(e, fused=True), st, cam, g, pixel_cost="ncc", refine=True, filt=True)
    steps = max(3, args.steps // 2)
    el, _ = timed(lambda: sp.run(rgbx), steps, max(1, args.warmup), e.device, world, sync)
    return {"workload": c["workload"], "value": round(V * W * H * steps / el / 1e6, 3), "unit": "Mpix/s",
            "ms_per_step": round(el * 1e3 / steps, 4), "steps": steps, "n_gpus": world, "scaling": "strong",
            "views_per_gpu": g.block[1] - g.block[0], "sweep": "fused NCC sweep + WTA"}


def cpu_baseline_sharded_crop(e, cfg, W=256, H=128, S=16):
    """C4's workload on a crop the oracle finishes in seconds: the same 8 x 4
    array, 5-nearest-neighbour lists and 128 hypotheses, 256 x 128 pixels, S =
    16 (a scene 0..15 px deep, so the shifts stay inside the crop), the whole
    pipeline: SLIC, extents, superpixel sweep, fused NCC 5x5 sweep + WTA,
    refinement, consistency filter.  The oracle's time is the CPU baseline; the
    same crop through the view-sharded pipeline on this GPU gives the depth L1
    of every map (tests/test_gpu_c4.py runs the same comparison)."""
    import torch

    from cl_multiview_stereo_amd import params, synth
    from cl_multiview_stereo_amd.distributed import EngineBackend, ShardedPipeline, ViewGather
    from cl_multiview_stereo_amd.engine import CameraArray
    from oracle import oracle as orc

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    os.environ["OMP_NUM_THREADS"] = str(threads)
    aw, ah = cfg["aw"], cfg["ah"]
    V = aw * ah
    stack, _ = synth.make_stack(W, H, aw, ah, 0, 15, 1.0, 0xC4)
    levels = params.disparity_levels(cfg["dmin"], cfg["dmax"], 1)
    vs, sn = params.flatten_subsets(params.nearest_neighbours(aw, ah, cfg["knn"]))
    st = params.Settings(spixl_size=S, array_width=aw, array_height=ah, min_disp=cfg["dmin"], max_disp=cfg["dmax"],
                         inc=1, bl_ratio=1.0, window=cfg["K"], cost="ncc")
    t0 = time.perf_counter()
    outs = [orc.slic(stack[v], S) for v in range(V)]
    lab = np.stack([o[0] for o in outs])
    sp = np.stack([o[1] for o in outs])
    lb = np.stack([o[2] for o in outs])
    rep = orc.boundary(sp, lb, S)
    sp = orc.sweep(lab, sp, rep, levels, vs, sn, aw, 1.0, S)
    q = orc.l8(lab)
    want = {"disp": np.stack([orc.wta(orc.ncc_volume(q, levels, vs, sn, aw, 1.0, cfg["K"], z), levels)[0]
                              for z in range(V)])}
    want["disp_refined"] = orc.refine(sp, lb, rep, vs, sn, aw, 1.0, S)["disp"]
    want["disp_filtered"] = orc.filt(want["disp_refined"], aw, 1.0, 1.0)[1]
    t_all = time.perf_counter() - t0
    cpu = {"value": round(V * W * H / t_all / 1e6, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
           "sample": f"C4's workload on a {W}x{H} crop ({V} reference views, {len(levels)} hypotheses x "
                     f"{cfg['knn']} nearest neighbours, S={S}, refinement + filter) on oracle/mvs_oracle.c, "
                     f"OpenMP x{threads}: {t_all:.1f}s",
           **_cpu_info()}
    cam = CameraArray(aw, 1.0, levels, vs, sn)
    pipe = ShardedPipeline(EngineBackend(e, fused=True), st, cam, ViewGather(V), pixel_cost="ncc", refine=True,
                           filt=True)
    out = pipe.run(torch.from_numpy(stack).to(e.device))
    torch.cuda.synchronize()
    l1 = {}
    for k, od in want.items():
        gd = getattr(out, k).cpu().numpy()
        l1[k] = {"value": float(np.abs(gd - od).mean()), "bit_exact": bool(np.array_equal(gd, od))}
    res = {"value": l1["disp_filtered"]["value"], "unit": "px (mean |d_gpu - d_oracle|)",
           "bit_exact": all(v["bit_exact"] for v in l1.values()), "map": "disp_filtered", "maps": l1,
           "sample": f"the same {W}x{H} crop through the view-sharded pipeline on this GPU (world 1), all {V} views"}
    return cpu, res


def cpu_baseline(pipe, stack, cfg, cost, out):
    """The oracle (CPU restatement, OpenMP) runs ONE full step of the same
    workload on this host: cvt + SLIC of every view, extents, the superpixel
    sweep, the per-pixel sweep + WTA of every reference view, and (C3 / ref)
    the refinement + fusion and the consistency filter.  At C2 that is ~10 s
    on 16 threads.  Returns (cpu_baseline, depth L1 of the timed GPU step's
    maps against the oracle's)."""
    import torch

    from oracle import oracle as orc

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    os.environ["OMP_NUM_THREADS"] = str(threads)
    W, H, S = cfg["W"], cfg["H"], cfg["S"]
    cam = pipe.cam
    V = stack.shape[0]
    t0 = time.perf_counter()
    outs = [orc.slic(stack[v], S) if S > 1 else orc.grid(stack[v], 1) for v in range(V)]
    lab_all = np.stack([o[0] for o in outs])
    sp = np.stack([o[1] for o in outs])
    lb = np.stack([o[2] for o in outs])
    rep = orc.boundary(sp, lb, S)
    sp = orc.sweep(lab_all, sp, rep, cam.levels, cam.view_subset, cam.subset_num, cfg["aw"], cfg["bl"], S)
    t_seg = time.perf_counter() - t0
    maps = {}
    rows, t_band = H, None
    if cost in ("ncc", "sad"):
        # the per-pixel sweep: a row band when the whole step would take the
        # host much longer than CPU_SAMPLE_SECONDS (SAD at D=128: ~160 s per
        # 1080p view per core; C5's NCC 7x7 at D=256: ~4 min on 16 threads).
        # With horizontal-only neighbours (every dy = 0) a pixel's window taps
        # and projections stay within rows y-R..y+R, so the band's rows above
        # its last R are exactly the full image's rows.
        horizontal = all(int(cam.view_subset[z, n]) // cfg["aw"] == z // cfg["aw"]
                         for z in range(V) for n in range(int(cam.subset_num[z])))
        K = cfg["K"] if cost == "ncc" else 5
        per_row = V * W * len(cam.levels) * max(1, int(cam.subset_num.max())) * K * K
        want = int(CPU_SAMPLE_SECONDS * CPU_TAP_RATE[cost] / per_row)
        rows = H if (not horizontal or want >= H) else max(64, want)
        lab_band = np.ascontiguousarray(lab_all[:, :rows])
        t1 = time.perf_counter()
        if cost == "ncc":
            q = orc.l8(lab_band)
            band = np.stack([orc.wta(orc.ncc_volume(q, cam.levels, cam.view_subset, cam.subset_num, cfg["aw"],
                                                    cfg["bl"], K, z), cam.levels)[0] for z in range(V)])
        else:
            band = orc.sweep_pixel_sad(lab_band, cam.levels, cam.view_subset, cam.subset_num, cfg["aw"], cfg["bl"])
        t_band = time.perf_counter() - t1
        keep = rows if rows == H else rows - K // 2
        maps["disp"] = (band[:, :keep], keep) if rows != H else band
    if cfg.get("refine"):
        maps["disp_refined"] = orc.refine(sp, lb, rep, cam.view_subset, cam.subset_num, cfg["aw"], cfg["bl"],
                                          S)["disp"]
        if cfg.get("filt"):
            maps["disp_filtered"] = orc.filt(maps["disp_refined"], cfg["aw"], cfg["bl"], 1.0)[1]
    t_all = time.perf_counter() - t0
    if rows != H:
        cpu = {"value": round(V * W * rows / t_band / 1e6, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
               "sample": f"the per-pixel {cost.upper()} sweep + WTA of rows 0..{rows - 1} of all {V} reference views "
                         f"({W} wide, "
                         f"{len(cam.levels)} hypotheses x {int(cam.subset_num.max())} neighbours) on "
                         f"oracle/mvs_oracle.c, OpenMP x{threads}: {t_band:.1f}s (segmentation of the full views, "
                         f"{t_seg:.1f}s, not counted)",
               **_cpu_info()}
    else:
        cpu = {"value": round(V * W * H / t_all / 1e6, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
               "sample": f"one full step of the bench workload ({V} reference views, {len(cam.levels)} hypotheses"
                         f"{', refinement' if cfg.get('refine') else ''}{', filter' if cfg.get('filt') else ''}) on "
                         f"oracle/mvs_oracle.c, OpenMP x{threads}: {t_all:.1f}s (segmentation + superpixel sweep "
                         f"{t_seg:.1f}s)",
               **_cpu_info()}
    torch.cuda.synchronize()
    l1 = {}
    sample = f"the last timed step's disparity maps, all {V} reference views, {W}x{H}"
    for k, od in maps.items():
        gd = getattr(out, k).cpu().numpy()
        if isinstance(od, tuple):  # a row band (the per-pixel sweep's sample)
            od, keep = od
            gd = gd[:, :keep]
            sample = (f"rows 0..{keep - 1} (the CPU sample's exact rows) of the last timed step's disparity maps, "
                      f"all {V} reference views, {W} wide")
        l1[k] = {"value": float(np.abs(gd - od).mean()), "bit_exact": bool(np.array_equal(gd, od))}
    head = "disp" if "disp" in l1 else ("disp_filtered" if "disp_filtered" in l1 else "disp_refined")
    res = {"value": l1[head]["value"], "unit": "px (mean |d_gpu - d_oracle|)", "bit_exact": l1[head]["bit_exact"],
           "map": head, "maps": l1, "sample": sample}
    return cpu, res


if __name__ == "__main__":
    main()
