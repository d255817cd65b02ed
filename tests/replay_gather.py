"""Gathers for measuring / testing the view-sharded pipeline on ONE GPU.

RecordingGather: ViewGather (world 1) that keeps every tensor it returns.
ReplayGather: stands in for ViewGather at (rank, world) with no
communication -- each gather returns the recorded world-1 tensor with the
rank's freshly computed block written into it, so the rank reads exactly the
neighbour data a real all-gather would deliver and does exactly its share of
the work (scripts/c4_shard_sim.py, tests/test_gpu_c4.py)."""
import torch

from cl_multiview_stereo_amd.distributed import ViewGather, all_blocks


class RecordingGather(ViewGather):
    def __init__(self, V):
        super().__init__(V)
        self.rec = []

    def __call__(self, local, full=None):
        out = super().__call__(local, full)
        self.rec.append(out.clone())
        return out

    def rows_to_views(self, rows_full):
        out = super().rows_to_views(rows_full)
        self.rec.append(out.clone())
        return out


class ReplayGather:
    """Stands in for ViewGather(V) at (rank, world): no communication."""

    def __init__(self, V, rank, world, rec):
        self.V, self.rank, self.world, self.rec = V, rank, world, rec
        self.blocks = all_blocks(V, world)
        self.i = 0
        self.bytes_in = 0
        self.narrow = {}     # recorded int32 labels as the bytes of their 16-bit values, made once
        self.events = None   # a list: (start, end) CUDA events around every replay copy

    @property
    def block(self):
        return self.blocks[self.rank]

    def start(self, local, full):
        from cl_multiview_stereo_amd.distributed import PendingGather
        return PendingGather(self(local, full))

    def __call__(self, local, full=None):
        z0, z1 = self.block
        rec = self.rec[self.i % len(self.rec)]
        if rec.dtype == torch.int32 and local.dtype == torch.uint8:
            # the world-1 run gathered the labels as int32; at world > 1 they
            # travel as the bytes of their 16-bit values (distributed._narrow_labels)
            k = self.i % len(self.rec)
            if k not in self.narrow:
                self.narrow[k] = rec.to(torch.int16).view(torch.uint8).view(rec.shape[0], -1)
            rec = self.narrow[k]
        self.i += 1
        self.bytes_in += (rec.numel() - local.numel()) * rec.element_size()
        ev = None
        if self.events is not None and rec.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        if full is None:
            full = rec.clone()
        elif full.data_ptr() != rec.data_ptr():
            full.copy_(rec)
        full[z0:z1] = local
        if ev is not None:
            ev[1].record()
            self.events.append(ev)
        return full

    def row_band(self, H):
        return all_blocks(H, self.world)[self.rank]

    def rows_to_views(self, rows_full):
        """The rows -> views exchange of the row-sharded filter: the rank's views,
        its own rows freshly computed, the other rows from the world-1 run."""
        z0, z1 = self.block
        ya, yb = self.row_band(rows_full.shape[1])
        rec = self.rec[self.i % len(self.rec)]
        self.i += 1
        ev = None
        if self.events is not None and rec.is_cuda:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        out = rec[z0:z1].clone()
        out[:, ya:yb] = rows_full[z0:z1, ya:yb]
        if ev is not None:
            ev[1].record()
            self.events.append(ev)
        self.bytes_in += (out.numel() - out[:, ya:yb].numel()) * out.element_size()
        return out

    def copy_ms(self):
        """Total device time of the replay copies recorded since events = [] (synchronise first):
        work a real all-gather into the caller's buffer does not add to the rank's stream."""
        return sum(a.elapsed_time(b) for a, b in (self.events or []))
