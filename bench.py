#!/usr/bin/env python3
"""Headline benchmark: Mpix/s of per-view depth on synthetic 5-view 1080p
stacks, 128 disparity hypotheses, NCC 5x5, SLIC K~2000 (BASELINE.json config 2).

One step = the whole depth pipeline over one batch: for each of the V reference
views of this rank's stack (inputs RGBx already resident in HBM): Lab
conversion, SLIC (S=32, 5 update/assign iterations), superpixel extents, the
reference superpixel SAD sweep, the per-pixel NCC 5x5 cost volume over 128
hypotheses x 4 neighbours and its winner-take-all + confidence pass.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2] [--cost ncc|sad]

N>1: launched by torch.distributed.run, one rank per GPU; every rank owns its
own 5-view stack (independent objects, no data-path collective) -> weak scaling.
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
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
                        "the GPUs (RCCL all-gathers of labels/spixl, refinement state, disparity)"),
    # the reference's own defaults (clMVDE.cpp main): its algorithm exactly, no per-pixel sweep
    "ref": dict(aw=3, ah=3, W=1920, H=1080, S=8, dmin=30, dmax=60, K=5, nh=1, nv=1, bl=1.0359, cost="none",
                refine=True,
                workload="clMVDE main() defaults: 3x3 array 1080p, S=8 (32,400 superpixels/view), levels 30..60, "
                         "superpixel SAD sweep + refinement (5 propagations) + fusion, all 9 views"),
    "c5": dict(aw=5, ah=1, W=4096, H=3072, S=40, dmin=0, dmax=255, K=7, nh=4, nv=0, bl=1.0, cost="ncc",
               workload="5-view 4096x3072, 256 hypotheses, NCC 7x7, SLIC K=7931 (S=40)"),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--cost", default=None, choices=["ncc", "sad", "none"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--concurrent", action="store_true",
                    help="superpixel chain on a second stream beside the per-pixel chain (pipeline.py)")
    ap.add_argument("--fused", action="store_true",
                    help="NCC sweep with the winner-take-all folded in (mvs_ncc_wta_d: no cost volume in HBM)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from cl_multiview_stereo_amd import params, synth
    from cl_multiview_stereo_amd.engine import Engine
    from cl_multiview_stereo_amd.pipeline import Pipeline

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    cfg = dict(CONFIGS[args.config])
    cost = args.cost or cfg["cost"]
    V = cfg["aw"] * cfg["ah"]
    W, H = cfg["W"], cfg["H"]
    st = params.Settings(spixl_size=cfg["S"], array_width=cfg["aw"], array_height=cfg["ah"], min_disp=cfg["dmin"],
                         max_disp=cfg["dmax"], inc=1, neib_hor=cfg["nh"], neib_ver=cfg["nv"], bl_ratio=cfg["bl"],
                         window=cfg["K"], cost=cost)
    D = cfg["dmax"] - cfg["dmin"] + 1

    e = Engine(local)
    sharded = bool(cfg.get("sharded"))
    # independent stacks per rank (weak scaling) or one array sharded by view (strong)
    stack, _ = synth.make_stack(W, H, cfg["aw"], cfg["ah"], cfg["dmin"], cfg["dmax"], cfg["bl"],
                                0x5EED + 2 + (0 if sharded else rank))
    rgbx = torch.from_numpy(stack).to(e.device)
    vlists = (params.nearest_neighbours(cfg["aw"], cfg["ah"], cfg["knn"]) if cfg.get("knn") else None)
    pipe = Pipeline(e, st, W, H, view_subset=vlists, pixel_cost=None if cost == "none" else cost,
                    refine=bool(cfg.get("refine")),
                    filt=bool(cfg.get("filt")) and not sharded, concurrent=args.concurrent, fused=args.fused)
    if sharded:
        from cl_multiview_stereo_amd.distributed import EngineBackend, ShardedPipeline, ViewGather
        spipe = ShardedPipeline(EngineBackend(e, fused=args.fused), st, pipe.cam, ViewGather(V), pixel_cost=cost, refine=True,
                                filt=bool(cfg.get("filt")))

    # HIP events around the cost-volume kernels, on the stream they run on
    timers = {"wta": [], "ncc": [], "fused": []}
    if pipe.pixel is not None and cost == "ncc":
        orig_wta, orig_vol = e.wta, e.ncc_volume

        def timed(name, fn):
            def w(*a, **k):
                s = torch.cuda.Event(enable_timing=True)
                t = torch.cuda.Event(enable_timing=True)
                s.record()
                r = fn(*a, **k)
                t.record()
                if timing[0]:
                    timers[name].append((s, t))
                return r
            return w
        timing = [False]
        e.wta = timed("wta", orig_wta)
        e.ncc_volume = timed("ncc", orig_vol)
        e.ncc_wta = timed("fused", e.ncc_wta)
    else:
        timing = [False]

    def step():
        return spipe.run(rgbx) if sharded else pipe.exe_pipeline(rgbx)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    timing[0] = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    timing[0] = False
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], device=e.device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    ms_per_step = elapsed * 1e3 / max(args.steps, 1)
    units = V if sharded else world * V  # reference views processed per step, whole job
    mpix = units * W * H * args.steps / elapsed / 1e6

    res = {
        "metric": "Mpix/s depth (1080p, 128 depth hyp, 5 views) + depth L1 vs ref",
        "value": round(mpix, 3),
        "unit": "Mpix/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "strong" if sharded else "weak",
        "vs_baseline": None,
        "dtype": "f32/i32",
        "data": "synthetic (seeded rendered camera-array stack, RGBx resident in HBM)",
        "config": {"workload": cfg["workload"], "views": V, "width": W, "height": H, "hypotheses": D,
                   "window": cfg["K"], "cost": cost, "spixl_size": cfg["S"],
                   "neighbours": int(pipe.cam.subset_num.max()),
                   "parallelism": (f"views sharded over {world} GPU(s)" if sharded else
                                   f"view-stack per GPU x{world}"),
                   "refinement": bool(cfg.get("refine")), "consistency_filter": bool(cfg.get("filt"))},
    }

    def avg(lst):
        return sum(s.elapsed_time(t) for s, t in lst) / len(lst) * 1e-3

    def valu_insts(fused):
        # SQ_INSTS_VALU per launch (profiles/pmc_ncc.json, C2), launch-weighted over
        # the band-width variants of the plain (FUSE=false) or fused kernel
        pmc_ncc = os.path.join(ROOT, "profiles", "pmc_ncc.json")
        if args.config != "c2" or cost != "ncc" or not os.path.exists(pmc_ncc):
            return None
        tag = "true>" if fused else "false>"
        ent = [v for k, v in json.load(open(pmc_ncc)).items() if k.startswith("k_ncc_volume") and k.endswith(tag)]
        if not ent:
            return None
        wts = [e.get("launches", 1) for e in ent]
        return sum(e["valu_wave_insts_per_launch"] * w for e, w in zip(ent, wts)) / sum(wts)

    VALU_PEAK = 1024 * 2.4e9 / 4.0  # wave64 VALU ops/s: 1024 SIMDs x 2.4 GHz / 4 cycles
    if args.fused and timers["fused"]:
        # no volume: the fused sweep is VALU-issue-bound
        t_ncc = avg(timers["fused"])
        insts = valu_insts(True)
        res["roofline"] = {"bound": "valu", "kernel": "k_ncc_volume<..., FUSE=true> (sweep + WTA, no volume)",
                           "achieved": None if insts is None else round(insts / t_ncc / 1e9, 1),
                           "peak": VALU_PEAK / 1e9, "unit": "G wave-instructions/s",
                           "frac": None if insts is None else round(insts / t_ncc / VALU_PEAK, 4),
                           "traffic": None, "avg_launch_ms": round(t_ncc * 1e3, 4)}
    if timers["wta"]:
        t_wta = avg(timers["wta"])
        t_ncc = avg(timers["ncc"])
        wta_bytes = 4.0 * D * W * H + 8.0 * W * H  # volume read + disparity/confidence write
        achieved = wta_bytes / t_wta / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_wta.json")
        if os.path.exists(pmc):
            try:
                traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        res["roofline"] = {"bound": "hbm", "kernel": "k_wta (cost-volume read pass)", "achieved": round(achieved, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                           "traffic": traffic, "algorithmic_bytes_per_launch": wta_bytes,
                           "avg_launch_ms": round(t_wta * 1e3, 4)}
        cells = float(D) * W * H
        nbr = max(1, int(pipe.cam.subset_num[0]))
        vol_bytes = 4.0 * cells
        res["roofline_sweep"] = {"kernel": "k_ncc_volume (cost-volume write pass)", "avg_launch_ms": round(t_ncc * 1e3, 4),
                                 "view_cells_per_s": round(cells * nbr / t_ncc / 1e9, 3),
                                 "unit_view_cells": "G view-cells/s",
                                 "hbm_write_GBps": round(vol_bytes / t_ncc / 1e9, 1),
                                 "hbm_write_frac": round(vol_bytes / t_ncc / 1e9 / HBM_PEAK_GBS, 4)}
        # VALU issue bound of the producer (its binding resource): wave-instructions per
        # launch from the SQ_INSTS_VALU pass (profiles/pmc_ncc.json, C2) at one
        # instruction per 4 cycles per SIMD, 1024 SIMDs, 2.4 GHz
        insts = valu_insts(False)
        if insts is not None:
            res["roofline_sweep"].update({"bound": "valu", "valu_wave_insts_per_launch": round(insts),
                                          "valu_issue_frac": round(insts / t_ncc / VALU_PEAK, 4),
                                          "valu_peak": "1024 SIMDs x 2.4 GHz / 4 cycles per wave64 op"})

    # the same step with the WTA folded into the sweep kernel (no cost volume in
    # HBM): timed with the same protocol after the headline run, outputs
    # compared bit-for-bit with the headline step's
    if cost == "ncc" and not args.fused and not sharded and not cfg.get("refine"):
        fpipe = Pipeline(e, st, W, H, view_subset=vlists, pixel_cost=cost, fused=True)
        for _ in range(max(1, args.warmup)):
            fout = fpipe.exe_pipeline(rgbx)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        timing[0] = True
        f0 = time.perf_counter()
        for _ in range(args.steps):
            fout = fpipe.exe_pipeline(rgbx)
        torch.cuda.synchronize()
        fel = time.perf_counter() - f0
        timing[0] = False
        if world > 1:
            dist.barrier()
            tt = torch.tensor([fel], device=e.device, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            fel = float(tt.item())
        same = bool(torch.equal(fout.disp.view(torch.int32), out.disp.view(torch.int32)) and
                    torch.equal(fout.conf.view(torch.int32), out.conf.view(torch.int32)))
        res["fused_variant"] = {"what": "bench.py --fused: k_ncc_volume with the WTA folded in, no cost volume in HBM",
                                "value": round(units * W * H * args.steps / fel / 1e6, 3), "unit": "Mpix/s",
                                "ms_per_step": round(fel * 1e3 / max(args.steps, 1), 4),
                                "bit_identical_to_headline": same,
                                "sweep_avg_launch_ms": round(avg(timers["fused"]) * 1e3, 4) if timers["fused"] else None}
        fi = valu_insts(True)
        if fi is not None and timers["fused"]:
            res["fused_variant"]["valu_issue_frac"] = round(fi / avg(timers["fused"]) / VALU_PEAK, 4)

    if rank == 0 and world == 1 and not args.no_cpu_baseline and (not cfg.get("refine") or cost == "none"):
        try:
            res["cpu_baseline"], res["depth_l1_vs_oracle"] = cpu_baseline(e, pipe, stack, cfg, cost, rgbx, out)
        except Exception as ex:  # report, never hide
            res["cpu_baseline"] = {"error": repr(ex)}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(e, pipe, stack, cfg, cost, rgbx, out):
    """The oracle (CPU restatement, OpenMP) runs ONE full step of the same
    workload on this host: cvt + SLIC of every view, extents, the superpixel
    sweep and the per-pixel sweep + WTA of every reference view.  At C2 that
    is ~10 s on 16 threads.  Returns (cpu_baseline, depth L1 of the timed GPU
    step's disparity maps against the oracle's, over all reference views)."""
    import torch

    from oracle import oracle as orc

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
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
    if cost == "none":  # the reference pipeline: refinement + fusion of every view
        od = orc.refine(sp, lb, rep, cam.view_subset, cam.subset_num, cfg["aw"], cfg["bl"], S)["disp"]
    elif cost == "ncc":
        q = orc.l8(lab_all)
        od = np.stack([orc.wta(orc.ncc_volume(q, cam.levels, cam.view_subset, cam.subset_num, cfg["aw"], cfg["bl"],
                                              cfg["K"], z), cam.levels)[0] for z in range(V)])
    else:
        od = orc.sweep_pixel_sad(lab_all, cam.levels, cam.view_subset, cam.subset_num, cfg["aw"], cfg["bl"])
    t_all = time.perf_counter() - t0
    cpu = {"value": round(V * W * H / t_all / 1e6, 4), "unit": "Mpix/s", "cores": threads, "kind": "port",
           "sample": f"one full step of the bench workload ({V} reference views, {len(cam.levels)} hypotheses) on "
                     f"oracle/mvs_oracle.c, OpenMP x{threads}: {t_all:.1f}s (segmentation+superpixel sweep "
                     f"{t_seg:.1f}s)"}
    torch.cuda.synchronize()
    gd = (out.disp_refined if cost == "none" else out.disp).cpu().numpy()
    l1 = float(np.abs(gd - od).mean())
    return cpu, {"value": l1, "unit": "px (mean |d_gpu - d_oracle|)", "bit_exact": bool(np.array_equal(gd, od)),
                 "sample": f"the last timed step's disparity maps, all {V} reference views, {W}x{H}"}


if __name__ == "__main__":
    main()
