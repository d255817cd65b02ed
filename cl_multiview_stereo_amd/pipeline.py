"""Host orchestration mirroring the reference's stage classes.

    SLIC              <- clSLIC              (clSLIC.cpp:67-122)
    PhotoConsistency  <- clPhotoConsistency  (photo_consistency.cpp:21-208)
    PixelSweep        <- build-defined per-pixel sweep (NCC KxK / SAD parity)
    DepthRefinement   <- clDepthRefinement   (depth_refinement.cpp:91-1470)
    ConsistencyFilter <- the reference's disabled fusion tail (1374-1453)
    Pipeline          <- pipeline            (pipeline.cpp:7-175)

All buffers live on the GPU for the whole run (HBM-resident stacks); every
stage is a HIP kernel in libmvs.so.  A Pipeline owns a contiguous block of
reference views [z0, z1) so one process per GPU can shard a large array by
reference view (see distributed.py).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import params
from .engine import CameraArray, Engine


class SLIC:
    """clSLIC: cvt + SLIC for a batch of views in one launch per kernel."""

    def __init__(self, engine: Engine, settings: params.Settings):
        self.e = engine
        self.st = settings

    def do_super_pixel_seg(self, rgbx: torch.Tensor):
        lab, l8 = self.e.cvt(rgbx, want_l8=True)
        spixl, labels = self.segment(lab)
        return lab, l8, spixl, labels

    def segment(self, lab: torch.Tensor):
        """The SLIC loop on converted views (everything after cvt)."""
        S = self.st.spixl_size
        if S == 1:
            return self.e.grid(lab, 1)
        return self.e.slic(lab, S, self.st.slic_color_weight, self.st.no_iter, self.st.enforce_connectivity,
                           search=self.st.slic_search)


class PhotoConsistency:
    """clPhotoConsistency::do_initial_depth_estimation: boundary + per-superpixel
    SAD plane sweep, one launch per reference view (photo_consistency.cpp:133)."""

    def __init__(self, engine: Engine, cam: CameraArray, S: int):
        self.e, self.cam, self.S = engine, cam, S

    def do_initial_depth_estimation(self, lab, spixl, labels, z0=0, z1=None):
        rep = self.e.boundary(spixl, labels, self.S)
        self.e.sweep_spixl(lab, spixl, rep, self.cam, self.S, z0, z1)
        return spixl, rep


class PixelSweep:
    """Per-pixel plane sweep.  cost="ncc": build-defined KxK NCC cost volume
    [D][H][W] per reference view, then WTA + confidence (the HBM-streaming
    pass); fused=True folds the WTA into the sweep kernel (mvs_ncc_wta_d: no
    volume in HBM, same disp/conf bits).  cost="sad": the reference sweep at
    S=1 grid semantics (parity)."""

    def __init__(self, engine: Engine, cam: CameraArray, W: int, H: int, cost: str = "ncc", window: int = 5,
                 fused: bool = False):
        self.e, self.cam, self.W, self.H = engine, cam, W, H
        self.cost, self.K, self.fused = cost, window, fused
        self.vol = None
        if cost == "ncc" and not fused:
            self.vol = engine.empty((cam.D, H, W), torch.float32)
        self.levels = engine.levels_dev(cam)

    def run(self, lab, l8, z0: int, z1: int, disp_out=None, conf_out=None, views=None):
        """Reference views [z0, z1).  views: the views whose window planes are
        built (default all; a view shard passes its block + neighbours)."""
        n = z1 - z0
        disp = self.e.empty((n, self.H, self.W), torch.float32) if disp_out is None else disp_out
        conf = None
        if self.cost == "sad":
            self.e.sweep_pixel_sad(lab, self.cam, z0, z1, out=disp)
            return disp, None
        conf = self.e.empty((n, self.H, self.W), torch.float32) if conf_out is None else conf_out
        if views is None:
            box = self.e.box_stats(l8, self.K)
        else:
            V, H, W = l8.shape
            box = self.e.box_stats_views(l8, self.K, views, self.e.empty((2, V, H + (H & 1), W, 2), torch.int32))
        if self.fused:  # every reference view of the call, runs of views per launch
            self.e.ncc_wta_range(l8, box, self.cam, z0, z1, self.K, disp=disp, conf=conf)
            return disp, conf
        for i, z in enumerate(range(z0, z1)):
            self.e.ncc_volume(l8, box, self.cam, z, self.K, out=self.vol)
            self.e.wta(self.vol, self.levels, disp=disp[i], conf=conf[i])
        return disp, conf


class DepthRefinement:
    """clDepthRefinement(...)->do_refinement(gamma, alpha, fuse, kernel_step,
    kernel_size, no_prop) + fusion (spixl_to_image)."""

    def __init__(self, engine: Engine, cam: CameraArray, S: int):
        self.e, self.cam, self.S = engine, cam, S

    def do_refinement(self, spixl, labels, rep, st: params.Settings, fusion_compat: bool = True):
        return self.e.refine(spixl, labels, rep, self.cam, self.S, st.gamma, st.alpha, st.fuse, st.kernel_step,
                             st.kernel_size, st.no_prop, fusion_compat)


class ConsistencyFilter:
    def __init__(self, engine: Engine, array_width: int, bl_ratio: float, fuse: float):
        self.e, self.aw, self.bl, self.fuse = engine, array_width, bl_ratio, fuse

    def run(self, disp_all: torch.Tensor, z0: int = 0, z1: int | None = None):
        return self.e.filter(disp_all, self.aw, self.bl, self.fuse, z0, z1)


@dataclass
class StepOutput:
    lab: torch.Tensor
    spixl: torch.Tensor
    labels: torch.Tensor
    rep: torch.Tensor
    disp: torch.Tensor | None = None
    conf: torch.Tensor | None = None
    disp_refined: torch.Tensor | None = None
    disp_filtered: torch.Tensor | None = None


class Pipeline:
    """pipeline: segmentation -> depth init -> [refinement] -> [filter].

    The reference's exe_pipeline runs SLIC only (perform_depth_est is commented
    out, pipeline.cpp:60-64); this pipeline wires the depth stages in the order
    of pipeline::perform_depth_est (pipeline.cpp:108-175).

    concurrent=True: after the colour conversion the superpixel chain (SLIC,
    extents, superpixel sweep: latency/L2-bound gathers) runs on a second HIP
    stream with its own libmvs context, beside the per-pixel chain (window
    planes, fused NCC sweep + WTA) on the caller's stream; the caller's stream
    joins the side stream before refinement.  One stream is the default here
    and in bench.py (round 5: with the matrix-core sweep the side stream
    measured no gain); `bench.py --concurrent` runs the headline
    with it, and the default line reports it as `concurrent_variant`."""

    def __init__(self, engine: Engine, settings: params.Settings, W: int, H: int,
                 view_subset: list[list[int]] | None = None, pixel_cost: str | None = "ncc",
                 refine: bool = False, filt: bool = False, concurrent: bool = False, fused: bool = False):
        self.e, self.st, self.W, self.H = engine, settings, W, H
        vs = view_subset if view_subset is not None else params.neighbour_lists(
            settings.array_width, settings.array_height, settings.neib_hor, settings.neib_ver)
        mat, num = params.flatten_subsets(vs)
        levels = params.disparity_levels(settings.min_disp, settings.max_disp, settings.inc)
        self.cam = CameraArray(settings.array_width, settings.bl_ratio, levels, mat, num)
        self.slic = SLIC(engine, settings)
        self.photo = PhotoConsistency(engine, self.cam, settings.spixl_size)
        self.pixel = PixelSweep(engine, self.cam, W, H, pixel_cost, settings.window, fused) if pixel_cost else None
        self.refiner = DepthRefinement(engine, self.cam, settings.spixl_size) if refine else None
        self.filter = ConsistencyFilter(engine, settings.array_width, settings.bl_ratio, settings.fuse) if filt else None
        self.side = None
        if concurrent and self.pixel is not None:
            side_engine = Engine(engine.device.index)  # own context: own scratch, metadata and plans
            self.side = (torch.cuda.Stream(engine.device), SLIC(side_engine, settings),
                         PhotoConsistency(side_engine, self.cam, settings.spixl_size))

    def exe_pipeline(self, rgbx: torch.Tensor, z0: int = 0, z1: int | None = None,
                     gather=None) -> StepOutput:
        """rgbx [V,H,W,4] resident on the GPU.  [z0, z1) = reference views this
        process owns; `gather` (distributed.py) all-gathers per-view maps."""
        V = rgbx.shape[0]
        z1 = V if z1 is None else z1
        if self.side is None:
            lab, l8, spixl, labels = self.slic.do_super_pixel_seg(rgbx)
            spixl, rep = self.photo.do_initial_depth_estimation(lab, spixl, labels, z0, z1)
            out = StepOutput(lab, spixl, labels, rep)
            if self.pixel is not None:
                out.disp, out.conf = self.pixel.run(lab, l8, z0, z1)
        else:
            lab, l8 = self.e.cvt(rgbx, want_l8=True)
            main = torch.cuda.current_stream(self.e.device)
            stream, slic, photo = self.side
            stream.wait_stream(main)
            with torch.cuda.stream(stream):
                spixl, labels = slic.segment(lab)
                spixl, rep = photo.do_initial_depth_estimation(lab, spixl, labels, z0, z1)
            lab.record_stream(stream)  # allocated on main, read on the side stream
            disp, conf = self.pixel.run(lab, l8, z0, z1)
            main.wait_stream(stream)
            for t in (spixl, labels, rep):  # allocated on the side stream, used on main from here
                t.record_stream(main)
            out = StepOutput(lab, spixl, labels, rep, disp, conf)
        if self.refiner is not None:
            r = self.refiner.do_refinement(spixl, labels, rep, self.st)
            out.disp_refined = r["disp"]
        if self.filter is not None:
            src = out.disp_refined if out.disp_refined is not None else out.disp
            full = src if src.shape[0] == V else (gather(src) if gather else None)
            if full is None:
                raise ValueError("filter over a view shard needs a gather function")
            out.disp_filtered = self.filter.run(full, z0, z1)[1][z0:z1]
        return out
