"""The C2 step (bench.py's default configuration, fused sweep, one stream) timed
three ways on one GPU: eager with the fused sweep's kernel timing off, eager
with it on (as bench.py's headline pass runs), and replayed from a HIP graph
(torch.cuda.CUDAGraph) captured from one eager step.  Interleaved rounds;
prints ms per step and whether the graph's outputs equal the eager step's.
    python scripts/probes/graph_step.py [--steps 20] [--rounds 3]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from cl_multiview_stereo_amd import params, synth  # noqa: E402
from cl_multiview_stereo_amd.engine import Engine  # noqa: E402
from cl_multiview_stereo_amd.pipeline import Pipeline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    sys.path.insert(0, ROOT)
    import bench
    cfg = dict(bench.CONFIGS["c2"])
    W, H = cfg["W"], cfg["H"]
    st = params.Settings(spixl_size=cfg["S"], array_width=cfg["aw"], array_height=cfg["ah"], min_disp=cfg["dmin"],
                         max_disp=cfg["dmax"], inc=1, neib_hor=cfg["nh"], neib_ver=cfg["nv"], bl_ratio=cfg["bl"],
                         window=cfg["K"], cost="ncc")
    e = Engine(0)
    stack, _ = synth.make_stack(W, H, cfg["aw"], cfg["ah"], cfg["dmin"], cfg["dmax"], cfg["bl"], 0x5EED + 2)
    rgbx = torch.from_numpy(stack).to(e.device)
    p = Pipeline(e, st, W, H, pixel_cost="ncc", fused=True)
    sync = torch.cuda.synchronize

    def eager():
        return p.exe_pipeline(rgbx)

    for _ in range(3):
        ref = eager()
    sync()
    # capture one step on a side stream (torch's capture protocol), replay on it
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        eager()  # (a warm step on the capture stream)
        sync()
        with torch.cuda.graph(g, stream=s):
            gout = p.exe_pipeline(rgbx)
    sync()
    g.replay()
    sync()
    same = all(torch.equal(getattr(gout, f).view(torch.int32), getattr(ref, f).view(torch.int32))
               for f in ("disp", "conf"))

    def run(fn):
        sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            fn()
        sync()
        return (time.perf_counter() - t0) * 1e3 / a.steps

    res = {"eager": [], "eager_ktime": [], "graph": []}
    for _ in range(a.rounds):
        res["eager"].append(round(run(eager), 4))
        e.set_kernel_timing(True)
        res["eager_ktime"].append(round(run(eager), 4))
        e.kernel_times()
        e.set_kernel_timing(False)
        res["graph"].append(round(run(g.replay), 4))
    print(json.dumps({"ms_per_step": res, "graph_outputs_equal_eager": same}))


if __name__ == "__main__":
    main()
