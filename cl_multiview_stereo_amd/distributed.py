"""View-sharded depth pipeline: one process per GPU, RCCL over xGMI.

SURVEY.md 8(e).  The array's reference views are split into contiguous
blocks, one block per rank (``view_block``).  The reference launches every
stage over all views at once (photo_consistency.cpp:133, depth_refinement.cpp
:738-889).  Each rank here runs the stages only for its block, and the ranks
exchange exactly what later stages read from other views:

  stage                             reads from other views    exchange
  --------------------------------  ------------------------  ---------------------------
  cvt (a1), block + its neighbours  -                         none (every rank holds the
                                                              RGBx stack; converts only
                                                              the views its block reads)
  SLIC (a2-a6), own block           -                         all-gather labels, issued
                                                              here and waited for only
                                                              before refinement: it runs
                                                              beside the sweeps below
  boundary (a8), own block          -                         none
  superpixel sweep (a9), own block  Lab of neighbours         all-gather spixl (s7 = seed),
                                                              after the per-pixel sweep
  per-pixel NCC + WTA, own block    l8 / window planes of     none until the filter
                                    neighbours (built for the
                                    block + neighbours only)
  flatness (a11)                    -                         none (all views, a few us)
  init state (a12), own block       neighbours' s7 / labels   all-gather state (S=32:
                                                              49 KB/view)
  propagate (a13) x no_prop         neighbours' state         all-gather state every
                                                              iteration
  fusion (a14), ALL views           every view's spixl,       none: each rank renders
                                    labels and state          every view from the
                                                              gathered spixl/labels/state
                                                              (no refinement: all-gather
                                                              the disparity maps)
  projection (a15 i), own ROWS of   all disparity maps        none
  every reference view
  removal (a15 ii), own rows of     the proj slices at the    rows -> views exchange of
  every reference view              pixel (same rows), all    the filtered maps (each rank
                                    disparity maps            receives its views' other
                                                              rows: 1/world of a gather)

The filter is sharded by image ROWS (filter_shard="rows", the default): every
rank holds all V disparity maps after the fusion, and the projection and the
removal at a pixel read only those maps and the proj slices at that pixel, so
a rank filters rows [y0, y1) of every reference view with no proj all-gather
(the reference-view form, filter_shard="views", all-gathers the block's proj
slices in row bands: ~7/8 of V x H x W x 4 bytes into every rank).  The
world-1-like grid (every reference of a row in flight together) also keeps
the removal's gathers as local as in the unsharded run.

The backend does the compute for one rank: ``EngineBackend`` (HIP kernels
through libmvs.so) on a GPU.  The tests substitute a CPU stand-in of the same
interface, so that this orchestration runs under gloo with world_size 2.
The collectives use ``all_gather_into_tensor`` (RCCL on ROCm; gloo also
implements it, so the CPU tests run the same branch) for equal blocks, in
place when the local block is a slice of the full tensor, and fall back to a
padded list all-gather when blocks are ragged.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist

from . import params


def view_block(V: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous balanced block [z0, z1) of reference views for `rank`: the
    first V % world ranks take one extra view."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(V, world)
    z0 = rank * base + min(rank, extra)
    return z0, z0 + base + (1 if rank < extra else 0)


def all_blocks(V: int, world: int) -> list[tuple[int, int]]:
    return [view_block(V, r, world) for r in range(world)]


class ViewGather:
    """All-gather of per-view blocks along dim 0 into a full [V, ...] tensor.

    With equal blocks this is one ``all_gather_into_tensor`` (in place when
    `local` is `full`'s own block).  Ragged blocks (V % world != 0) use the
    padded list form."""

    def __init__(self, V: int, group=None):
        self.V = V
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.blocks = all_blocks(V, self.world)
        self.equal = len({z1 - z0 for z0, z1 in self.blocks}) == 1
        self.backend = dist.get_backend(group) if dist.is_initialized() else "none"

    @property
    def block(self) -> tuple[int, int]:
        return self.blocks[self.rank]

    def row_band(self, H: int) -> tuple[int, int]:
        """This rank's rows [y0, y1) of a row-sharded stage (balanced contiguous)."""
        return all_blocks(H, self.world)[self.rank]

    def rows_to_views(self, rows_full: torch.Tensor) -> torch.Tensor:
        """rows_full [V, H, W] holds this rank's row band of every view; returns
        [z1 - z0, H, W]: every row of this rank's view block.  Rank s sends rank d
        the rows of d's views in s's band (point to point, batched: RCCL groups
        them; gloo has no all_to_all)."""
        V, H = rows_full.shape[:2]
        z0, z1 = self.block
        if self.world == 1:
            return rows_full[z0:z1]
        bands = all_blocks(H, self.world)
        ya, yb = bands[self.rank]
        out = rows_full.new_empty((z1 - z0,) + tuple(rows_full.shape[1:]))
        out[:, ya:yb] = rows_full[z0:z1, ya:yb]
        ops, recv = [], []
        for d in range(self.world):
            if d == self.rank:
                continue
            b0, b1 = self.blocks[d]
            send = rows_full[b0:b1, ya:yb].contiguous()
            r0, r1 = bands[d]
            buf = rows_full.new_empty((z1 - z0, r1 - r0) + tuple(rows_full.shape[2:]))
            ops.append(dist.P2POp(dist.isend, send, d, group=self.group))
            ops.append(dist.P2POp(dist.irecv, buf, d, group=self.group))
            recv.append((r0, r1, buf, send))
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        for r0, r1, buf, _ in recv:
            out[:, r0:r1] = buf
        return out

    def start(self, local: torch.Tensor, full: torch.Tensor) -> "PendingGather":
        """The same all-gather, asynchronous: the collective is issued behind the
        work already on the current stream, later work on the stream runs beside
        it, and PendingGather.wait() makes the stream wait for it.  `local`
        must be `full`'s own block (in place)."""
        z0, z1 = self.block
        if local.shape[0] != z1 - z0 or full.shape[0] != self.V:
            raise ValueError(f"rank {self.rank}: bad block / full shapes")
        if self.world == 1 or not self.equal:
            return PendingGather(self(local, full))
        if local.data_ptr() != full[z0:z1].data_ptr():
            full[z0:z1] = local
        work = dist.all_gather_into_tensor(full, full[z0:z1], group=self.group, async_op=True)
        return PendingGather(full, work)

    def __call__(self, local: torch.Tensor, full: torch.Tensor | None = None) -> torch.Tensor:
        z0, z1 = self.block
        if local.shape[0] != z1 - z0:
            raise ValueError(f"rank {self.rank}: local block has {local.shape[0]} views, expected {z1 - z0}")
        shape = (self.V,) + tuple(local.shape[1:])
        if full is None:
            full = torch.empty(shape, dtype=local.dtype, device=local.device)
        if self.world == 1:
            if full.data_ptr() != local.data_ptr():
                full.copy_(local)
            return full
        if self.equal:
            src = local if local.is_contiguous() else local.contiguous()
            dist.all_gather_into_tensor(full, src, group=self.group)
            return full
        n_max = max(b1 - b0 for b0, b1 in self.blocks)
        pad_shape = (n_max,) + tuple(local.shape[1:])
        send = torch.zeros(pad_shape, dtype=local.dtype, device=local.device)
        send[:z1 - z0] = local
        bufs = [torch.empty(pad_shape, dtype=local.dtype, device=local.device) for _ in range(self.world)]
        dist.all_gather(bufs, send, group=self.group)
        for (b0, b1), buf in zip(self.blocks, bufs):
            full[b0:b1] = buf[:b1 - b0]
        return full


class PendingGather:
    def __init__(self, full: torch.Tensor, work=None):
        self.full, self.work = full, work

    def wait(self) -> torch.Tensor:
        if self.work is not None:
            self.work.wait()
            self.work = None
        return self.full


def _narrow_labels(g: ViewGather, spixl: torch.Tensor) -> bool:
    """Gather the labels as 16-bit values: more than one rank, and every label
    (< mw * mh) fits.  MVS_LABELS16=0 keeps the 32-bit gather (A/B)."""
    mw_mh = spixl.shape[1] * spixl.shape[2]
    return g.world > 1 and mw_mh <= 1 << 16 and os.environ.get("MVS_LABELS16", "1") != "0"


def _bytes(t: torch.Tensor) -> torch.Tensor:
    """A contiguous [n, ...] tensor as [n, bytes per view] uint8 (every
    collective backend moves bytes, gloo included)."""
    return t.view(torch.uint8).view(t.shape[0], -1)


def _expand(blk: torch.Tensor, V: int, z0: int) -> torch.Tensor:
    """[V, ...] holding `blk` at views [z0, z0 + len(blk)); the other views are
    left unset (an all-gather fills them before any stage reads them)."""
    full = blk.new_empty((V,) + tuple(blk.shape[1:]))
    full[z0:z0 + blk.shape[0]] = blk
    return full


@dataclass
class ShardOutput:
    z0: int
    z1: int
    spixl: torch.Tensor                 # [V, mh, mw, 8] (gathered, s7 = seed disparity)
    labels: torch.Tensor                # [V, H, W]      (gathered; int32, or uint16 after a narrowed gather)
    disp: torch.Tensor | None = None    # [z1-z0, H, W] per-pixel NCC/SAD disparity
    conf: torch.Tensor | None = None
    disp_refined: torch.Tensor | None = None   # [z1-z0, H, W]
    disp_filtered: torch.Tensor | None = None  # [z1-z0, H, W]

    def labels32(self) -> torch.Tensor:
        """The gathered labels as int32 (uint32 bits), widening 16-bit maps."""
        return self.labels if self.labels.dtype == torch.int32 else self.labels.to(torch.int32)


class ShardedPipeline:
    """pipeline::perform_segmentation + perform_depth_est (pipeline.cpp:60-175)
    over one rank's view block.  `backend` supplies the per-rank compute (see
    EngineBackend for the interface)."""

    def __init__(self, backend, settings: params.Settings, cam, gather: ViewGather,
                 pixel_cost: str | None = "ncc", refine: bool = True, filt: bool = True, proj_bands: int | None = None,
                 filter_shard: str | None = None):
        self.b, self.st, self.cam, self.g = backend, settings, cam, gather
        self.pixel_cost, self.refine, self.filt = pixel_cost, refine, filt
        # row bands of the pipelined proj all-gather of the reference-view
        # sharded filter (1: one gather; default: 2 when there is a gather to
        # hide, i.e. world > 1)
        self.proj_bands = proj_bands if proj_bands is not None else (2 if gather.world > 1 else 1)
        # "rows" (default; MVS_FILTER_SHARD overrides) or "views"
        self.filter_shard = filter_shard or os.environ.get("MVS_FILTER_SHARD", "rows")
        if self.filter_shard not in ("rows", "views"):
            raise ValueError("filter_shard must be 'rows' or 'views'")

    def run(self, rgbx: torch.Tensor) -> ShardOutput:
        st, b, g = self.st, self.b, self.g
        V = rgbx.shape[0]
        if V != g.V:
            raise ValueError("stack size does not match the gather's view count")
        z0, z1 = g.block
        S = st.spixl_size
        need = self.cam.views_needed(z0, z1)
        lab, l8 = b.cvt(rgbx, need)
        sp_blk, lb_blk = b.slic(lab[z0:z1], S, st.slic_color_weight, st.no_iter, st.enforce_connectivity,
                                st.slic_search)
        spixl = _expand(sp_blk, V, z0)
        labels = _expand(lb_blk, V, z0)
        # the labels (the largest gather) are read from other views only by the
        # refinement: in flight while this rank sweeps its block.  With fewer
        # than 2^16 superpixels per view they travel as 16-bit values (half the
        # bytes over xGMI), and the refinement and fusion kernels
        # read them as they arrive (no widening pass).
        narrow = _narrow_labels(g, spixl)
        if narrow:
            l16 = torch.empty(labels.shape, dtype=torch.int16, device=labels.device)
            l16[z0:z1] = lb_blk.to(torch.int16)  # two's-complement wrap keeps the low 16 bits
            pending = g.start(_bytes(l16[z0:z1]), _bytes(l16))
        else:
            pending = g.start(labels[z0:z1], labels)
        rep = b.boundary(spixl, labels, S, z0, z1)  # own block only
        b.sweep_spixl(lab, spixl, rep, self.cam, S, z0, z1)
        out = ShardOutput(z0, z1, spixl, labels)
        if self.pixel_cost:
            out.disp, out.conf = b.pixel_sweep(lab, l8, self.cam, z0, z1, self.pixel_cost, st.window, need)
        out.spixl = g(spixl[z0:z1], spixl)  # centres + seeds (s7) of every view
        if narrow:
            pending.wait()
            out.labels = l16.view(torch.uint16)
        else:
            out.labels = pending.wait()
        spixl, labels = out.spixl, out.labels
        full = None
        if self.refine:
            full = self._refine(spixl, labels, rep, z0, z1)
            out.disp_refined = full[z0:z1]
        if self.filt:
            if full is None:
                full = g(out.disp)
            out.disp_filtered = self._filter(full, z0, z1)
        return out

    def _filter(self, full, z0, z1):
        if self.filter_shard == "rows":
            return self._filter_rows(full)
        return self._filter_views(full, z0, z1)

    def _filter_rows(self, full):
        """project_to_reference_inv + remove_view_inconsistency (clcode.cl:1995-2101)
        for this rank's rows of EVERY reference view: the projection reads only
        the disparity maps, which every rank holds, and the removal at a pixel
        reads the proj slices at that pixel, which this rank has just computed.
        Then each rank receives the other rows of its own views."""
        st, b, g = self.st, self.b, self.g
        aw, bl, fuse = st.array_width, st.bl_ratio, st.fuse
        V, H, W = full.shape
        ya, yb = g.row_band(H)
        buf = full.new_empty((V, yb - ya, W))
        b.proj_inv(full, aw, bl, 0, V, proj=buf, rows=(ya, yb), band=True)
        res = full.new_empty(full.shape)  # only rows [ya, yb) are written
        res = b.remove_inconsistency(full, buf, aw, bl, fuse, 0, V, out=res, rows=(ya, yb), band=True)
        return g.rows_to_views(res)

    def _filter_views(self, full, z0, z1):
        """project_to_reference_inv for the block, then every rank holds all proj
        slices, which remove_view_inconsistency reads (clcode.cl:2054).  The
        removal at a pixel reads the proj slices at that pixel only, so with
        proj_bands > 1 the proj all-gather goes in row bands: band c's gather
        is issued as soon as its rows are projected and runs beside the next
        bands' projection and the earlier bands' removal."""
        st, b, g = self.st, self.b, self.g
        aw, bl, fuse = st.array_width, st.bl_ratio, st.fuse
        V, H, W = full.shape
        nb = max(1, min(self.proj_bands, H))
        res = full.new_empty(full.shape)  # only the block's views are written
        if nb == 1:
            proj = b.proj_inv(full, aw, bl, z0, z1)
            g(proj[z0:z1], proj)
            return b.remove_inconsistency(full, proj, aw, bl, fuse, z0, z1, out=res)[z0:z1]
        edges = [(H * i // nb, H * (i + 1) // nb) for i in range(nb)]
        bands = []
        for ya, yb in edges:  # the block's rows are projected straight into the band's gather buffer
            buf = full.new_empty((V, yb - ya, W))
            b.proj_inv(full, aw, bl, z0, z1, proj=buf, rows=(ya, yb), band=True)
            bands.append((ya, yb, buf, g.start(buf[z0:z1], buf)))
        for ya, yb, buf, pending in bands:  # the removal reads each gathered band in place
            res = b.remove_inconsistency(full, pending.wait(), aw, bl, fuse, z0, z1, out=res, rows=(ya, yb), band=True)
        return res[z0:z1]

    def _refine(self, spixl, labels, rep, z0, z1):
        """clDepthRefinement::do_refinement (depth_refinement.cpp:91-118, 724-889)
        with the Jacobi ping-pong of mvs_refine_d: the block's initial state
        and each iteration's output block are all-gathered before the next
        iteration reads the neighbours' states."""
        st, b, g = self.st, self.b, self.g
        rp = params.refine_params(st)
        flat = b.flatness(spixl, rp["flat_gamma"])
        state = b.init_state(spixl, labels, rep, flat, self.cam, st.spixl_size, rp["init_gamma"], rp["init_alpha"],
                             rp["kernel_steps"], rp["kss"], rp["fuse"], z0, z1)
        g(state[z0:z1], state)
        state2 = state.clone()
        for it in range(st.no_prop):
            src, dst = (state, state2) if it % 2 == 0 else (state2, state)
            nks, kss = params.prop_schedule(it, rp["kernel_steps"], rp["kss"])
            b.propagate(spixl, labels, rep, flat, self.cam, st.spixl_size, it, rp["prop_alpha"], rp["prop_gamma"],
                        rp["fuse"], nks, kss, src, dst, z0, z1)
            g(dst[z0:z1], dst)
        # fusion renders current_state_dev = `state` (Appendix A #13).  Every
        # rank holds every view's spixl, labels and `state` (gathered after
        # iteration 3), and a fused map is a function of those alone, so each
        # rank renders ALL views itself (~0.1 ms at C4) instead of all-gathering
        # the block's maps (8.3 MB per view: 232 MB into every rank at C4).
        return b.spixl_to_image(spixl, labels, state, st.spixl_size)


class EngineBackend:
    """Per-rank compute on the GPU through libmvs.so (Engine).  fused: the per-pixel
    NCC sweep folds its winner-take-all in (no cost volume; same maps).
    Buffers that only the listed views fill (Lab, l8, window planes, rep,
    state) are full-size [V, ...] so kernels index them by global view id."""

    def __init__(self, engine, fused: bool = False):
        self.e, self.fused = engine, fused
        self._sweeps = {}  # PixelSweep (volume buffers, side stream) per configuration

    def cvt(self, rgbx, views):
        V, H, W, _ = rgbx.shape
        lab = self.e.empty((V, H, W, 4), torch.float32)
        l8 = self.e.empty((V, H, W), torch.uint8)
        return self.e.cvt_views(rgbx, views, lab, l8)

    def slic(self, lab_blk, S, weight, no_iter, conn, search=0):
        if S == 1:
            return self.e.grid(lab_blk, 1)
        return self.e.slic(lab_blk, S, weight, no_iter, conn, search=search)

    def boundary(self, spixl, labels, S, z0, z1):
        rep = torch.zeros(tuple(spixl.shape[:3]) + (8,), dtype=torch.uint8, device=self.e.device)
        rep[z0:z1] = self.e.boundary(spixl[z0:z1], labels[z0:z1], S)
        return rep

    def sweep_spixl(self, lab, spixl, rep, cam, S, z0, z1):
        self.e.sweep_spixl(lab, spixl, rep, cam, S, z0, z1)

    def pixel_sweep(self, lab, l8, cam, z0, z1, cost, K, views):
        from .pipeline import PixelSweep
        H, W = lab.shape[1:3]
        key = (id(cam), W, H, cost, K)
        ps = self._sweeps.get(key)
        if ps is None:
            ps = self._sweeps[key] = PixelSweep(self.e, cam, W, H, cost, K, self.fused)
        return ps.run(lab, l8, z0, z1, views=views)

    def flatness(self, spixl, gamma):
        return self.e.flatness(spixl, gamma)

    def init_state(self, spixl, labels, rep, flat, cam, S, gamma, alpha, nks, kss, fuse, z0, z1):
        return self.e.init_state_range(spixl, labels, rep, flat, cam, S, gamma, alpha, nks, kss, fuse, z0, z1)

    def propagate(self, *a):
        return self.e.propagate(*a)

    def spixl_to_image(self, spixl, labels, state, S):
        return self.e.spixl_to_image(spixl.contiguous(), labels.contiguous(), state.contiguous(), S)

    def proj_inv(self, disp_full, aw, bl, z0, z1, proj=None, rows=None, band=False):
        return self.e.proj_inv(disp_full, aw, bl, z0, z1, proj=proj, rows=rows, band=band)

    def remove_inconsistency(self, disp_full, proj, aw, bl, fuse, z0, z1, out=None, rows=None, band=False):
        return self.e.remove_inconsistency(disp_full, proj, aw, bl, fuse, z0, z1, out=out, rows=rows, band=band)


def init_from_env(backend: str = "nccl"):
    """torch.distributed init for `torch.distributed.run` launches (RANK,
    LOCAL_RANK, WORLD_SIZE, MASTER_ADDR/PORT from the environment)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if backend == "nccl":
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return rank, world, local
