"""End-to-end run on the reference's own camera-array images.

The reference's main() (clMVDE/clMVDE.cpp:14-36) runs its pipeline on
Images/Beer-Garden/img0..8.png (3x3 array, data.txt), S=8, levels 30..60,
bl_ratio 1.0359, and plots the fused maps as 8-bit PNGs
(depth_refinement.cpp:1473-1495); results/8- Fusion/"fus4 <k>.png" are the 9
plots of that array it keeps (the fus1..fus3 sets have 15 views: another
array).  The parameters behind those plots are not recorded anywhere in the
reference, so they are compared as images, not as a parity oracle.

Three steps (this is checker infrastructure under tests/, not a pytest module):

  python tests/beer_garden.py prepare   # container: copy the 9 inputs into data/beer_garden/
  python tests/beer_garden.py gpu       # GPU box: mvs_cli on them (timed), the CPU oracle on
                                        # the same decoded pixels, bit-compare the depth maps
  python tests/beer_garden.py compare   # container: our fus <k>.png vs the reference's fus4 <k>.png

data/ is listed in .gpurunignore (it is 30 MB and only this script reads it):
take that line out for the `gpu` step.  The GPU step writes gpurun_out/beer/{result.json, fus <k>.png, init <k>.png};
`compare` writes profiles/archive/r02_beer_garden.json.  data/ is git-ignored: the
images are the reference's input data, not part of this repository's history.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
DATA = os.path.join(ROOT, "data", "beer_garden")
OUT = os.path.join(ROOT, "gpurun_out", "beer")
CLI = os.path.join(ROOT, "cl_multiview_stereo_amd", "mvs_cli")
REF_IMAGES = "/root/reference/Images/Beer-Garden"
REF_FUSION = "/root/reference/results/8- Fusion"
# clMVDE.cpp:14-36
AW, AH, S, DMIN, DMAX, BL = 3, 3, 8, 30, 60, 1.0359


def prepare():
    os.makedirs(DATA, exist_ok=True)
    names = [f"img{k}.png" for k in range(AW * AH)]
    for n in names:
        shutil.copyfile(os.path.join(REF_IMAGES, n), os.path.join(DATA, n))
    with open(os.path.join(DATA, "data.txt"), "w") as f:
        f.write("\n".join(names) + "\n")
    print("copied", len(names), "images to", DATA)


def _decode(path):
    """RGBx bytes through mvs_cli's loader (tested against an independent
    encoder for every colour type and filter in tests/test_host_cli.py)."""
    with tempfile.NamedTemporaryFile(suffix=".raw") as t:
        r = subprocess.run([CLI, "--png-decode", path, t.name], capture_output=True, text=True, check=True)
        W, H = map(int, r.stdout.split())
        return np.fromfile(t.name, np.uint8).reshape(H, W, 4)


def gpu():
    from cl_multiview_stereo_amd import params
    from oracle import oracle as orc

    os.makedirs(OUT, exist_ok=True)
    work = tempfile.mkdtemp(prefix="beer_")
    t0 = time.perf_counter()
    r = subprocess.run([CLI, "--data", os.path.join(DATA, "data.txt"), "--array", f"{AW}x{AH}", "--dump-init",
                        "--out", work], capture_output=True, text=True)
    t_cli = time.perf_counter() - t0
    if r.returncode != 0:
        raise SystemExit(f"mvs_cli failed: {r.stderr}")
    V = AW * AH
    for k in range(V):
        for p in (f"fus {k}.png", f"init {k}.png"):
            shutil.copyfile(os.path.join(work, p), os.path.join(OUT, p))
    stack = np.stack([_decode(os.path.join(DATA, f"img{k}.png")) for k in range(V)])
    H, W = stack.shape[1:3]
    depth = np.fromfile(os.path.join(work, "depth.f32"), np.float32).reshape(V, H, W)

    # the oracle, same settings (the reference's main() defaults)
    t1 = time.perf_counter()
    outs = [orc.slic(stack[v], S) for v in range(V)]
    lab = np.stack([o[0] for o in outs])
    sp = np.stack([o[1] for o in outs])
    lb = np.stack([o[2] for o in outs])
    rep = orc.boundary(sp, lb, S)
    levels = params.disparity_levels(DMIN, DMAX, 1)
    vs, sn = params.flatten_subsets(params.neighbour_lists(AW, AH, 1, 1))
    sp = orc.sweep(lab, sp, rep, levels, vs, sn, AW, BL, S)
    ref = orc.refine(sp, lb, rep, vs, sn, AW, BL, S)
    t_orc = time.perf_counter() - t1
    od = ref["disp"]
    per_view = []
    for v in range(V):
        per_view.append({"view": v, "bit_exact": bool(np.array_equal(depth[v].view(np.uint32), od[v].view(np.uint32))),
                         "l1": float(np.abs(depth[v] - od[v]).mean()),
                         "sha256_gpu": hashlib.sha256(depth[v].tobytes()).hexdigest()[:16],
                         "sha256_oracle": hashlib.sha256(od[v].tobytes()).hexdigest()[:16]})
    res = {"images": "reference Images/Beer-Garden img0..8.png (3x3 array, data.txt)", "W": W, "H": H,
           "settings": {"spixl_size": S, "levels": [DMIN, DMAX], "bl_ratio": BL, "neib": [1, 1], "no_iter": 5,
                        "gamma": 2, "alpha": 6, "fuse": 1, "kernel_size": 1080, "kernel_step": 13, "no_prop": 5},
           "mvs_cli_wall_s": round(t_cli, 3), "mvs_cli_stdout": r.stdout.strip().splitlines(),
           "oracle_wall_s": round(t_orc, 3), "oracle_threads": os.environ.get("OMP_NUM_THREADS"),
           "depth_bit_exact_all_views": all(p["bit_exact"] for p in per_view),
           "depth_l1_vs_oracle": float(np.mean([p["l1"] for p in per_view])), "per_view": per_view}
    with open(os.path.join(OUT, "result.json"), "w") as f:
        json.dump(res, f, indent=1)
    shutil.rmtree(work, ignore_errors=True)
    print(json.dumps({k: res[k] for k in ("mvs_cli_wall_s", "oracle_wall_s", "depth_bit_exact_all_views",
                                          "depth_l1_vs_oracle")}))


def compare():
    from pngio import read_png_gray

    res = json.load(open(os.path.join(OUT, "result.json")))
    rows = []
    for k in range(AW * AH):
        ours = read_png_gray(os.path.join(OUT, f"fus {k}.png")).astype(np.int32)
        theirs = _decode(os.path.join(REF_FUSION, f"fus4 {k}.png"))[..., 0].astype(np.int32)
        d = np.abs(ours - theirs)
        rows.append({"view": k, "equal": float((d == 0).mean()), "within_1": float((d <= 1).mean()),
                     "within_4": float((d <= 4).mean()), "within_16": float((d <= 16).mean()),
                     "mean_abs_grey": float(d.mean()),
                     "corr": float(np.corrcoef(ours.ravel(), theirs.ravel())[0, 1])})
    summ = {k: float(np.mean([r[k] for r in rows])) for k in ("equal", "within_1", "within_4", "within_16",
                                                               "mean_abs_grey", "corr")}
    out = {"what": "8-bit fused-depth plots of the reference's Beer-Garden array: ours (mvs_cli, the reference's "
                   "main() defaults) vs the reference's results/8- Fusion/'fus4 <k>.png'. The reference does not "
                   "record the parameters or code revision behind those plots, so this is an image comparison, "
                   "not a parity oracle; parity is the GPU-vs-oracle bit comparison in 'gpu_run'.",
           "summary": summ, "per_view": rows, "gpu_run": res}
    p = os.path.join(ROOT, "profiles", "r02_beer_garden.json")
    with open(p, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(summ))


if __name__ == "__main__":
    {"prepare": prepare, "gpu": gpu, "compare": compare}[sys.argv[1]]()
