#!/usr/bin/env python3
"""Isolated SLIC timing at C5's shape (5 views 4096x3072, S = 40) and the
reference defaults' (9 views 1080p, S = 8): min / median ms over 5 runs."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cl_multiview_stereo_amd import synth  # noqa: E402
from cl_multiview_stereo_amd.engine import Engine  # noqa: E402


def timeit(fn, reps=5):
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    return round(min(ts), 4), round(float(np.median(ts)), 4)


e = Engine(0)
out = {}
for name, (W, H, aw, ah, S) in {"c5_S40": (4096, 3072, 5, 1, 40), "ref_S8": (1920, 1080, 3, 3, 8)}.items():
    stack, _ = synth.make_stack(W, H, aw, ah, 0, 31, 1.0, 0x5EED + 2)
    lab, _ = e.cvt(torch.from_numpy(stack).cuda())
    e.slic(lab, S)
    torch.cuda.synchronize()
    out[name] = timeit(lambda: e.slic(lab, S))
print(json.dumps(out), flush=True)
