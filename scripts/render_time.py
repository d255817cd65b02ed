#!/usr/bin/env python3
"""Isolated spixl_to_image timing at C4's shape (32 views 1080p, S = 32, 16-bit
labels, as every rank of the view-sharded C4 runs it): min / median ms."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cl_multiview_stereo_amd import params  # noqa: E402
from cl_multiview_stereo_amd.engine import Engine  # noqa: E402

e = Engine(0)
V, W, H, S = 32, 1920, 1080, 32
mw, mh = params.map_size(W, H, S)
g = torch.Generator().manual_seed(7)
# labels: each pixel's own cell or a neighbour one, in runs as SLIC makes them
ys, xs = torch.meshgrid(torch.arange(H), torch.arange(W), indexing="ij")
jx = ((xs + 7 * (ys // 5)) % 41 > 35).long()
lab = ((ys // S) * mw + torch.clamp(xs // S + jx, max=mw - 1)).to(torch.int16)
labels = lab.expand(V, H, W).contiguous().cuda().view(torch.uint16)
spixl = torch.rand((V, mh, mw, 8), generator=g).cuda() * 30
state = torch.rand((V, mh, mw, 6), generator=g).cuda() + 0.5
out = e.spixl_to_image(spixl, labels, state, S)
ts = []
for _ in range(7):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    e.spixl_to_image(spixl, labels, state, S)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print(json.dumps({"render_32views_ms": [round(min(ts), 4), round(float(np.median(ts)), 4)],
                  "checksum": float(out.double().sum())}), flush=True)
