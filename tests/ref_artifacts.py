#!/usr/bin/env python3
"""Reconcile the oracle with the outputs the reference keeps in its tree.

The reference has no tests; the only record of what its OpenCL path
computed is the 8-bit PNGs under /root/reference/results/, written by its own
plot functions from real camera-array images under /root/reference/Images/.
This script re-renders each family the way the reference's writer does, from
the oracle's output on the same decoded pixels, and scores the agreement over
a documented grid of settings.  CPU only, container only (the reference tree
does not exist on the GPU box); it lives under tests/ because it loads the
oracle.  Writes profiles/archive/r03_ref_artifacts.json.

Renderers (reference file:line):
  * SLIC overlay  -- clSLIC::draw_segmentation_lines, clSLIC.cpp:447-478: an
    interior pixel (1..H-2, 1..W-2) is painted when its label differs from one
    of its 4 neighbours, else copied from the input; the border rows/columns
    are never written (the overlays hold MSVC's 0xCD fill there) and are not
    scored.  The reference mask is "overlay pixel != input pixel".
  * seed plot     -- clPhotoConsistency::img_translate, photo_consistency.cpp:414-437:
    floor((s7 - 30) / 30 * 255) of the pixel's superpixel.
  * state plot    -- clDepthRefinement::img_translate_state, depth_refinement.cpp:1498-1553
    (element 0, range 30..60), written after propagate iteration 4 (:804-809).
  * fusion plot   -- plot_full_image, depth_refinement.cpp:1473-1495, of the
    fused disparity (spixl_to_image of current_state_dev, :1352).
  * flatness plot -- img_translate_flatness, depth_refinement.cpp:299-322: ceil(fl.s0 * 255).
  An 8-bit store of an out-of-range value is taken modulo 256 (MSVC x64
  converts through a 32-bit integer).

Settings grid (SLIC): candidate search (0 = the active 2x2 loop,
clcode.cl:474-494; 1 = the 3x3 loop behind the comment switch at :496-516),
no_iter, enforce_connectivity, colour weight; S = 8 (main(), clMVDE.cpp:15).
Numerical variants: the pinned oracle (SLIC centre means as x * RN(1/n)), the
contracting build (clang -ffp-contract=on -mfma, oracle/Makefile `contract`)
and the IEEE-quotient probe (`probe`: x / n, this build's definition before
round 3).

    python tests/ref_artifacts.py [--quick]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from cl_multiview_stereo_amd import params  # noqa: E402
from oracle import oracle as orc  # noqa: E402

REF = "/root/reference"
BUILDS = {"pinned": orc.LIB_PATH,
          "contract": os.path.join(ROOT, "oracle", "_build", "liboracle_contract.so"),
          "ieeediv": os.path.join(ROOT, "oracle", "_build", "liboracle_ieeediv.so")}
F32 = np.float32

# input sets: the 5x3 array (Images/c<k>f1.png) and the 3x3 Beer-Garden array
C_SCENE = [f"Images/c{k}f1.png" for k in range(15)]
BEER = [f"Images/Beer-Garden/img{k}.png" for k in range(9)]
OVERLAYS = [  # family, input set, overlay path pattern
    ("blue", C_SCENE, "results/blue{k}.png"),
    ("blue_i", C_SCENE, "results/blue_i{k}.png"),
    ("con_i", C_SCENE, "results/slic output/con_i{k}.png"),
    ("green", BEER, "results/slic output/green{k}.png"),
    ("green_new", BEER, "results/slic output/green_new{k}.png"),
    ("green_new_2", BEER, "results/slic output/green_new_2{k}.png"),
]


def use(build):
    orc._lib = C.CDLL(BUILDS[build])


def load_rgb(rel):
    from PIL import Image  # container-only dependency of this script
    return np.array(Image.open(os.path.join(REF, rel)).convert("RGB"))


def load_gray(rel):
    from PIL import Image
    a = np.array(Image.open(os.path.join(REF, rel)))
    return a if a.ndim == 2 else a[..., 0]


def rgbx_of(rgb):
    out = np.zeros(rgb.shape[:2] + (4,), np.uint8)
    out[..., :3] = rgb  # loadImageIn, file_handler.cpp:6-14: s0 = R
    return out


def boundary_mask(labels):
    """draw_segmentation_lines' test, clSLIC.cpp:458-461 (interior only)."""
    lb = labels.astype(np.int64)
    m = np.zeros(lb.shape, bool)
    c = lb[1:-1, 1:-1]
    m[1:-1, 1:-1] = (c != lb[1:-1, 2:]) | (c != lb[1:-1, :-2]) | (c != lb[:-2, 1:-1]) | (c != lb[2:, 1:-1])
    return m


def overlay_mask(overlay, rgb):
    return ~(overlay == rgb).all(-1)


INNER = np.s_[1:-1, 1:-1]


def plot8(d, lo=30.0, hi=60.0):
    v = np.floor(((d.astype(F32) - F32(lo)) / (F32(hi) - F32(lo))) * F32(255))
    return (v.astype(np.int64) % 256).astype(np.uint8)


def per_pixel(spixl_field, labels):
    return spixl_field.reshape(-1)[labels.astype(np.int64)].reshape(labels.shape)


# ---------------------------------------------------------------------------
def score_overlays(quick):
    out = {}
    grid = [(s, it, conn, w) for s in (0, 1) for it in ((1, 5) if quick else (0, 1, 2, 3, 5))
            for conn in (0, 1) for w in ((0.6,) if quick else (0.6, 0.3, 1.0))]
    for fam, inputs, pat in OVERLAYS:
        rgb0 = load_rgb(inputs[0])
        ref0 = overlay_mask(load_rgb(pat.format(k=0)), rgb0)
        use("pinned")
        res = []
        for s, it, conn, w in grid:
            _, _, lb = orc.slic(rgbx_of(rgb0), 8, w, it, conn, search=s)
            mism = int(np.count_nonzero(boundary_mask(lb)[INNER] != ref0[INNER]))
            res.append({"search": s, "no_iter": it, "connectivity": conn, "weight": w,
                        "view0_mismatch_px": mism, "view0_agreement": 1 - mism / ref0[INNER].size})
        res.sort(key=lambda r: r["view0_mismatch_px"])
        best = res[0]
        views = range(len(inputs)) if not quick else range(min(3, len(inputs)))
        per_build = {}
        for build in ("pinned", "contract", "ieeediv"):
            use(build)
            per = []
            for k in views:
                rgb = load_rgb(inputs[k])
                ref = overlay_mask(load_rgb(pat.format(k=k)), rgb)
                _, _, lb = orc.slic(rgbx_of(rgb), 8, best["weight"], best["no_iter"], best["connectivity"],
                                    search=best["search"])
                per.append(int(np.count_nonzero(boundary_mask(lb)[INNER] != ref[INNER])))
            n = len(per) * ref0[INNER].size
            per_build[build] = {"mismatch_px_per_view": per, "mismatch_px": sum(per),
                                "agreement": 1 - sum(per) / n}
        use("pinned")
        out[fam] = {"inputs": inputs[0].rsplit("/", 1)[0] + "/", "overlay": pat, "views": len(list(views)),
                    "reference_overlay_fraction": float(ref0[INNER].mean()),
                    "best_setting": {k: best[k] for k in ("search", "no_iter", "connectivity", "weight")},
                    "best_all_views": per_build, "grid_view0": res[:8]}
        print(f"[overlay] {fam}: best {out[fam]['best_setting']} -> "
              f"{per_build['pinned']['mismatch_px']} px of {n} ({per_build['pinned']['agreement']:.7f})", flush=True)
    return out


# ---------------------------------------------------------------------------
def beer_garden_stack(search, build="pinned"):
    use(build)
    st = params.Settings()  # main()'s defaults: 3x3, S 8, levels 30..60, bl 1.0359
    labs, sps, lbs = [], [], []
    for k in range(9):
        lab, sp, lb = orc.slic(rgbx_of(load_rgb(BEER[k])), st.spixl_size, st.slic_color_weight, st.no_iter,
                               st.enforce_connectivity, search=search)
        labs.append(lab)
        sps.append(sp)
        lbs.append(lb)
    lab, sp, lb = np.stack(labs), np.stack(sps), np.stack(lbs)
    rep = orc.boundary(sp, lb, st.spixl_size)
    levels = params.disparity_levels(st.min_disp, st.max_disp, st.inc)
    vs, sn = params.flatten_subsets(params.neighbour_lists(st.array_width, st.array_height, st.neib_hor,
                                                           st.neib_ver))
    sp = orc.sweep(lab, sp, rep, levels, vs, sn, st.array_width, st.bl_ratio, st.spixl_size)
    return dict(lab=lab, spixl=sp, labels=lb, rep=rep, vs=vs, sn=sn, st=st)


def purity(labels, plot):
    """Fraction of pixels whose grey equals the most common grey of their
    superpixel: 1.0 iff the plot is constant on every superpixel of `labels`."""
    key = labels.astype(np.int64) * 256 + plot
    u, c = np.unique(key, return_counts=True)
    best = np.zeros(int(labels.max()) + 1, np.int64)
    np.maximum.at(best, u // 256, c)
    return float(best.sum() / plot.size)


def reference_seeds(spixl, labels):
    """The reference's own seeds, read back from initD_dev<k>.png: the plot is
    injective on the integer levels 30..60, and constant on each superpixel."""
    levels = np.arange(30, 61, dtype=F32)
    grey = plot8(levels)
    inv = {int(g): float(l) for g, l in zip(grey, levels)}
    sp = spixl.copy()
    changed = 0
    for k in range(sp.shape[0]):
        g = load_gray(f"results/1- initialize disparity/initD_dev{k}.png").astype(np.int64)
        lb = labels[k].astype(np.int64)
        key = lb * 256 + g
        u, c = np.unique(key, return_counts=True)
        order = np.lexsort((-c, u // 256))
        u = u[order]
        first = np.unique(u // 256, return_index=True)[1]
        ids, gv = u[first] // 256, u[first] % 256
        flat = sp[k].reshape(-1, 8)
        new = np.array([inv.get(int(x), np.nan) for x in gv], F32)
        ok = ~np.isnan(new)
        changed += int(np.count_nonzero(flat[ids[ok], 7] != new[ok]))
        flat[ids[ok], 7] = new[ok]
    return sp, changed


def score_depth(quick):
    out = {}
    stacks = {}
    for search in (0, 1):
        t0 = time.time()
        b = beer_garden_stack(search)
        stacks[search] = b
        eq, pur = [], []
        for k in range(9):
            ref = load_gray(f"results/1- initialize disparity/initD_dev{k}.png")
            ours = plot8(per_pixel(b["spixl"][k][..., 7], b["labels"][k]))
            eq.append(float((ours == ref).mean()))
            pur.append(purity(b["labels"][k], ref))
        out[f"seeds_search{search}"] = {"plot": "results/1- initialize disparity/initD_dev<k>.png",
                                        "equal_frac_per_view": eq, "equal_frac": float(np.mean(eq)),
                                        "reference_plot_constant_on_our_superpixels": float(np.mean(pur)),
                                        "seconds": time.time() - t0}
        print(f"[seeds] search {search}: equal {np.mean(eq):.5f}, purity {np.mean(pur):.5f}", flush=True)
    b = stacks[1]
    st = b["st"]
    ref_sp, changed = reference_seeds(b["spixl"], b["labels"])
    for seeds, sp in (("ours", b["spixl"]), ("reference", ref_sp)):
        for build in (("pinned",) if quick else ("pinned", "contract")):
            use(build)
            r = orc.refine(sp, b["labels"], b["rep"], b["vs"], b["sn"], st.array_width, st.bl_ratio, st.spixl_size,
                           st.gamma, st.alpha, st.fuse, st.kernel_step, st.kernel_size, st.no_prop)
            it4, fus = [], []
            for k in range(9):
                g = load_gray(f"results/7- propagate/change6_alter1 {k}.png")
                it4.append(float((plot8(per_pixel(r["states"][4][k][..., 0], b["labels"][k])) == g).mean()))
                f = load_gray(f"results/8- Fusion/fus4 {k}.png")
                fus.append(float((plot8(r["disp"][k]) == f).mean()))
            out[f"refine_{seeds}_seeds_{build}"] = {
                "state_iter4_plot_equal_frac": float(np.mean(it4)), "per_view_state_iter4": it4,
                "fus4_plot_equal_frac": float(np.mean(fus)), "per_view_fus4": fus}
            print(f"[refine] {seeds} seeds, {build}: iter-4 state {np.mean(it4):.4f}, fus4 {np.mean(fus):.4f}",
                  flush=True)
    out["reference_seeds_changed"] = changed
    out["superpixels"] = int(b["spixl"][..., 7].size)
    use("pinned")
    return out


def score_flatness(quick):
    out = {}
    ks = range(3) if quick else range(15)
    for search in (0, 1):
        eq, w1 = [], []
        for k in ks:
            _, sp, lb = orc.slic(rgbx_of(load_rgb(C_SCENE[k])), 8, search=search)
            fl = orc.flatness(sp[None], 1.0 / 8.0)[0]  # gamma' = 2 * 2^2 (pipeline.cpp:164), 1/gamma' (:130)
            ours = (np.ceil(per_pixel(fl[..., 0], lb) * F32(255)).astype(np.int64) % 256)
            ref = load_gray(f"results/2- flatness/flatness_new {k}.png").astype(np.int64)
            eq.append(float((ours == ref).mean()))
            w1.append(float((np.abs(ours - ref) <= 1).mean()))
        out[f"search{search}"] = {"equal_frac": float(np.mean(eq)), "within_1_frac": float(np.mean(w1)),
                                  "views": len(list(ks))}
        print(f"[flatness] search {search}: equal {np.mean(eq):.4f}, within 1 {np.mean(w1):.4f}", flush=True)
    return out


# ---------------------------------------------------------------------------
# Refinement sensitivity (round 4): how far does each implementation-defined
# choice move the refinement, against how far the reference's own plots sit?
PROBE_BUILDS = {  # oracle/Makefile `probes`, MVS_PROBE_* in oracle/mvs_oracle.c
    "rcpdiv": "every fp32 quotient of the refinement as a * RN(1/b)",
    "libmexp": "glibc exp/expf in place of mvs_detmath",
    "expulp1": "every expf result moved by a hash-chosen -1..+1 ulp",
    "expulp2": "every expf result moved by a hash-chosen -2..+2 ulp",
    "sqrtrsq": "sqrt(s) as s * RN(1/sqrt(s))",
    "rcontract": "mul+add contracted (FMA) in the refinement only",
    "rsys": "the systematic alternatives together: rcpdiv + libmexp + sqrtrsq + rcontract",
    "rall": "all of the above together (ulp 1)",
    # other draws of the ulp hash (one draw is a sample, not a bound)
    "expulp1s1": "expf -1..+1 ulp, hash seed 1", "expulp1s2": "expf -1..+1 ulp, hash seed 2",
    "expulp1s3": "expf -1..+1 ulp, hash seed 3", "expulp2s1": "expf -2..+2 ulp, hash seed 1",
    "expulp2s2": "expf -2..+2 ulp, hash seed 2", "expulp2s3": "expf -2..+2 ulp, hash seed 3",
}


def perturb_labels(labels, n, seed):
    """Flip n interior boundary pixels of one view to the label of a 4-neighbour
    that differs (the size of the reference's residual SLIC disagreement)."""
    rng = np.random.default_rng(seed)
    lb = labels.copy()
    m = boundary_mask(lb)
    ys, xs = np.nonzero(m)
    pick = rng.choice(len(ys), size=min(n, len(ys)), replace=False)
    for y, x in zip(ys[pick], xs[pick]):
        nb = [lb[y + dy, x + dx] for dy, dx in ((0, 1), (0, -1), (1, 0), (-1, 0)) if lb[y + dy, x + dx] != lb[y, x]]
        if nb:
            lb[y, x] = nb[rng.integers(len(nb))]
    return lb


def refine_plots(sp, lb, rep, b):
    st = b["st"]
    r = orc.refine(sp, lb, rep, b["vs"], b["sn"], st.array_width, st.bl_ratio, st.spixl_size, st.gamma, st.alpha,
                   st.fuse, st.kernel_step, st.kernel_size, st.no_prop)
    it4 = np.stack([plot8(per_pixel(r["states"][4][k][..., 0], lb[k])) for k in range(9)])
    fus = np.stack([plot8(r["disp"][k]) for k in range(9)])
    return it4, fus


def score_probes(label_flips=46):
    """Started from the reference's seeds (read back from initD_dev<k>), the
    refinement of every probe build and of label-perturbed inputs, each scored
    against the reference's plots (7- propagate iteration 4, 8- Fusion fus4)
    and against the pinned oracle's own plots; plus where the pinned oracle's
    fus4 disagreement with the reference lies, bucketed by the distance to the
    nearest pixel where its SLIC boundary differs from the reference's
    (slic output/green<k>.png, the search-1 overlay family)."""
    from scipy import ndimage
    for name in PROBE_BUILDS:
        BUILDS[name] = os.path.join(ROOT, "oracle", "_build", f"liboracle_{name}.so")
        if not os.path.exists(BUILDS[name]):
            os.system(f"make -s -C {os.path.join(ROOT, 'oracle')} probes")
    b = beer_garden_stack(1)
    ref_sp, _ = reference_seeds(b["spixl"], b["labels"])
    ref_it4 = np.stack([load_gray(f"results/7- propagate/change6_alter1 {k}.png") for k in range(9)])
    ref_fus = np.stack([load_gray(f"results/8- Fusion/fus4 {k}.png") for k in range(9)])
    out = {"start": "the reference's seeds on the pinned oracle's search-1 labels", "variants": {}}

    def record(name, what, it4, fus, base=None):
        e = {"what": what, "iter4_vs_reference": float((it4 == ref_it4).mean()),
             "fus4_vs_reference": float((fus == ref_fus).mean())}
        if base is not None:
            e["iter4_vs_pinned"] = float((it4 == base[0]).mean())
            e["fus4_vs_pinned"] = float((fus == base[1]).mean())
        out["variants"][name] = e
        print(f"[probe] {name:12s} ref: it4 {e['iter4_vs_reference']:.4f} fus4 {e['fus4_vs_reference']:.4f}"
              + (f"   pinned: it4 {e['iter4_vs_pinned']:.4f} fus4 {e['fus4_vs_pinned']:.4f}" if base else ""),
              flush=True)

    t0 = time.time()
    use("pinned")
    base = refine_plots(ref_sp, b["labels"], b["rep"], b)
    record("pinned", "the pinned definition", *base)
    out["seconds_per_refinement"] = time.time() - t0
    for name, what in PROBE_BUILDS.items():
        use(name)
        record(name, what, *refine_plots(ref_sp, b["labels"], b["rep"], b), base=base)
    # (d) labels perturbed at label_flips boundary pixels per view (~the
    # reference's 412 SLIC residual pixels over the 9 views).  The superpixel
    # records stay: SLIC's last step is an assignment, so the centres and
    # colours the refinement reads are the previous labels' means (re-averaging
    # them from the final labels moves every superpixel, not a few).  The
    # extents are recomputed from the perturbed labels.
    S = b["st"].spixl_size
    for build in ("pinned", "rall"):
        for seed in (1, 2):
            use("pinned")
            lbp = np.stack([perturb_labels(b["labels"][k], label_flips, 1000 * seed + k) for k in range(9)])
            repp = orc.boundary(ref_sp, lbp, S)
            use(build)
            record(f"labels{seed}" + ("" if build == "pinned" else "+rall"),
                   f"{label_flips} boundary pixels per view flipped (seed {seed})"
                   + ("" if build == "pinned" else "; " + PROBE_BUILDS["rall"]),
                   *refine_plots(ref_sp, lbp, repp, b), base=base)
    use("pinned")
    # where the pinned oracle leaves the reference's fus4 plot
    ref_mask = np.stack([overlay_mask(load_rgb(f"results/slic output/green{k}.png"), load_rgb(BEER[k]))
                         for k in range(9)])
    ours = np.stack([boundary_mask(b["labels"][k]) for k in range(9)])
    edges = [0, 4, 16, 64, 256, 1 << 30]
    hist = {f"{lo}-{hi}" if hi < 1 << 30 else f">={lo}": [0, 0] for lo, hi in zip(edges, edges[1:])}
    sp_dis = []
    for k in range(9):
        mism = np.zeros(ours[k].shape, bool)
        mism[INNER] = ours[k][INNER] != ref_mask[k][INNER]
        dist = ndimage.distance_transform_edt(~mism) if mism.any() else np.full(mism.shape, np.inf)
        bad = base[1][k] != ref_fus[k]
        for (lo, hi), key in zip(zip(edges, edges[1:]), hist):
            sel = (dist >= lo) & (dist < hi)
            hist[key][0] += int(sel.sum())
            hist[key][1] += int((bad & sel).sum())
        lbk = b["labels"][k].astype(np.int64)
        n_sp = int(lbk.max()) + 1
        bad_sp = np.bincount(lbk.ravel(), weights=bad.ravel(), minlength=n_sp)
        tot_sp = np.bincount(lbk.ravel(), minlength=n_sp)
        sp_dis.append(((bad_sp > 0).sum(), (bad_sp >= 0.5 * np.maximum(tot_sp, 1)).sum(), (tot_sp > 0).sum()))
    out["fus4_disagreement_by_distance_to_slic_mismatch"] = {
        k: {"pixels": v[0], "disagreeing": v[1], "frac": v[1] / max(v[0], 1)} for k, v in hist.items()}
    sp_dis = np.array(sp_dis).sum(0)
    out["fus4_disagreement_superpixels"] = {"any_pixel": int(sp_dis[0]), "majority": int(sp_dis[1]),
                                           "superpixels": int(sp_dis[2])}
    print("[probe] disagreement by distance to a SLIC mismatch:",
          {k: round(v["frac"], 4) for k, v in out["fus4_disagreement_by_distance_to_slic_mismatch"].items()})
    return out


STAGE_PLOTS = {  # the per-superpixel stage plots of the 15-view c<k>f1 array
    "flatness_new": "results/2- flatness/flatness_new {k}.png",
    "initSm_dev": "results/3- initialize smoothness/initSm_dev {k}.png",
    "initCs_dev": "results/4- initialize consistency/initCs_dev {k}.png",
}


def score_stage_purity():
    """Whether the flatness / init-smoothness / init-consistency plots come
    from the same SLIC labels as the oracle's: each plot is a per-superpixel
    value painted over the superpixel's pixels (depth_refinement.cpp:299-322,
    390-391), so on the labels that made it the plot is constant on every
    superpixel (purity 1.0, as the seed plots are on the oracle's labels:
    99.9986 %).  A purity well below 1 on the oracle's labels (both
    candidate searches) means another run's segmentation, so these plots
    cannot pin the oracle's flatness / init stages."""
    out = {}
    for fam, pat in STAGE_PLOTS.items():
        row = {}
        for search in (0, 1):
            pur = []
            for k in range(15):
                _, _, lb = orc.slic(rgbx_of(load_rgb(C_SCENE[k])), 8, search=search)
                pur.append(purity(lb, load_gray(pat.format(k=k))))
            row[f"search{search}"] = {"purity": float(np.mean(pur)), "per_view": pur}
        out[fam] = row
        print(f"[purity] {fam}: search 0 {row['search0']['purity']:.4f}, search 1 {row['search1']['purity']:.4f}",
              flush=True)
    # the reference: the seed plots of the Beer-Garden array on the oracle's labels
    b = beer_garden_stack(1)
    pur = [purity(b["labels"][k], load_gray(f"results/1- initialize disparity/initD_dev{k}.png")) for k in range(9)]
    out["initD_dev (Beer-Garden, control)"] = {"search1": {"purity": float(np.mean(pur)), "per_view": pur}}
    print(f"[purity] control initD_dev: {np.mean(pur):.6f}", flush=True)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--purity", action="store_true",
                    help="only the stage-plot purity check (profiles/r04/ref_stage_purity.json)")
    ap.add_argument("--quick", action="store_true", help="fewer views and settings (about a minute)")
    ap.add_argument("--probes", action="store_true",
                    help="only the refinement sensitivity table (profiles/r04/ref_probes.json)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if not os.path.isdir(REF):
        sys.exit("ref_artifacts: /root/reference is absent (container-only script)")
    if a.purity:
        res = score_stage_purity()
        out = a.out or os.path.join(ROOT, "profiles", "r04", "ref_stage_purity.json")
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
        print("wrote", out)
        return
    if a.probes:
        res = score_probes()
        out = a.out or os.path.join(ROOT, "profiles", "r05", "ref_probes.json")
        with open(out, "w") as f:
            json.dump(res, f, indent=1)
        print("wrote", out)
        return
    a.out = a.out or os.path.join(ROOT, "profiles", "r03_ref_artifacts.json")
    for b, path in BUILDS.items():
        if not os.path.exists(path):
            os.system(f"make -s -C {os.path.join(ROOT, 'oracle')} {'all' if b == 'pinned' else b}")
    t0 = time.time()
    res = {"what": "oracle vs the reference's kept PNG outputs (tests/ref_artifacts.py)",
           "overlays": score_overlays(a.quick), "depth_beer_garden": score_depth(a.quick),
           "flatness_c_scene": score_flatness(a.quick), "quick": a.quick}
    res["seconds"] = time.time() - t0
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", a.out)


if __name__ == "__main__":
    main()
