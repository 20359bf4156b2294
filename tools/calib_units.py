#!/usr/bin/env python3
"""Calibrate the executed-work model's unit costs (rtg_amd/work.py UNIT_COST)
against the hardware's count of issued VALU instructions (VERDICT r04 item 1:
the model read 3.5 % above PMC on C3).

GPU part (`--collect DIR`, run under rocprofv3 --pmc SQ_INSTS_VALU): renders a
set of scenes of both kernel kinds (masked scenes of <= 64 spheres, BVH
scenes above) once with the default kernel and once with its counting build
(variant 120), and writes DIR/scenes.json with the counting build's per-unit
wave counts in render order.  The PMC record of the k-th default-kernel trace
dispatch is scene k's SQ_INSTS_VALU.

CPU part (`--fit DIR`): solves for unit costs c >= 0 minimising the relative
residuals of  sum_u waves[k, u] c_u  against SQ_INSTS_VALU[k], with a ridge
toward the source-priced costs (so units the scene set does not separate keep
their prices), and prints the fitted table and the per-scene residuals before
and after, plus held-out ratios for the bench configs (each left out of its
own fit; and a fit on the seeded scenes alone).  The prior and the 0.6-1.7x
bounds are always the source prices (work.py UNIT_COST_SOURCE), so a refit
never starts from an earlier fit.

  rocprofv3 --pmc SQ_INSTS_VALU --output-format csv -d OUT -o run -- \\
      python3 tools/calib_units.py --collect OUT
  python3 tools/calib_units.py --fit OUT
  python3 tools/calib_units.py --fit profiles/r06/calib_units   # the committed data
"""
import argparse
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def scenes(rng):
    """(name, spheres, lights, W, H, S) of the calibration set."""
    import rtg_amd as R
    from conftest import random_scene
    from bench import CONFIGS
    out = []
    for c, (W, H, n, m, depth) in sorted(CONFIGS.items()):
        sph, lg = R.generate_scene(n, m)
        # the bench configs at full size (C4 at half, C5 at a quarter of each side):
        # the fit is judged on the bench lines' model/PMC ratio
        f = {"c4": 2, "c5": 4}.get(c, 1)
        out.append((c, sph, lg, max(64, W // f), max(48, H // f), depth + 1))
    for k in range(14):  # masked scenes (n <= 64)
        n, m = int(rng.integers(2, 65)), int(rng.integers(1, 5))
        sph, lg = random_scene(rng, n, m)
        out.append((f"mask{k}", sph, lg, 480, 270, int(rng.integers(2, 9))))
    for k in range(10):  # BVH scenes: generator clusters of 65..600 spheres
        n, m = int(rng.integers(65, 601)), int(rng.integers(1, 5))
        sph, lg = R.generate_scene(n, m, seed=1000 + k)
        out.append((f"bvh{k}", sph, lg, 480, 270, int(rng.integers(3, 9))))
    return out


def collect(out_dir):
    import torch
    import rtg_amd as R
    os.makedirs(out_dir, exist_ok=True)
    rng = np.random.default_rng(77)
    ctx = R.Context(0)
    st = torch.cuda.current_stream()
    rec = []
    for name, sph, lg, W, H, S in scenes(rng):
        ctx.set_scene(sph, lg)
        fb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        ctx.set_variant(0)
        ctx.render_device(W, H, fb.data_ptr(), stack_size=S, stream=st.cuda_stream)
        torch.cuda.synchronize()
        ctx.set_variant(120)
        ctx.diag_counts(reset=True)
        ctx.render_device(W, H, fb.data_ptr(), stack_size=S, stream=st.cuda_stream)
        torch.cuda.synchronize()
        wv, lv = ctx.diag_counts(reset=True)
        ctx.set_variant(0)
        rec.append({"scene": name, "n": len(sph), "m": len(lg), "W": W, "H": H, "S": S,
                    "waves": {nm: int(wv[k]) for k, nm in enumerate(R.UNIT_NAMES)}})
        print(name, len(sph), W, H, S, flush=True)
    json.dump(rec, open(os.path.join(out_dir, "scenes.json"), "w"))
    ctx.close()


def load_pmc(d):
    rows = []
    js = os.path.join(d, "pmc.json")  # the committed form (profiles/r06/calib_units/)
    if os.path.exists(js):
        for r in json.load(open(js)):
            nm = r["kernel"]
            if "Li120E" in nm or ", 120," in nm:
                continue
            rows.append((r["dispatch"], r["SQ_INSTS_VALU"]))
        rows.sort()
        return [v for _, v in rows]
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != "SQ_INSTS_VALU":
                continue
            nm = r["Kernel_Name"]
            if "trace_samples_kernel" not in nm or "Li120E" in nm or ", 120," in nm:
                continue
            rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    rows.sort()
    return [v for _, v in rows]


def solve(A, y, wgt, c0, lam):
    """Unit costs c in [0.6, 1.7] x c0 minimising the weighted relative
    residuals of A c against y, with a ridge (relative) toward c0."""
    from scipy.optimize import lsq_linear
    Ar = A / y[:, None] * wgt[:, None]
    reg = np.sqrt(lam) * np.diag(1.0 / c0)
    M = np.vstack([Ar, reg])
    b = np.concatenate([wgt, np.sqrt(lam) * np.ones(len(c0))])
    return lsq_linear(M, b, bounds=(0.6 * c0, 1.7 * c0)).x


def fit(d, lam):
    # The prior and the bounds are the SOURCE prices (rtg_amd/work.py
    # UNIT_COST_SOURCE), never a previous fit's, so refits do not drift.
    from rtg_amd.work import UNIT_COST_SOURCE
    bench = ("c2", "c3", "c4", "c5")
    rec = json.load(open(os.path.join(d, "scenes.json")))
    y = np.array(load_pmc(d))
    assert len(y) == len(rec), (len(y), len(rec))
    units = [u for u in UNIT_COST_SOURCE if any(r["waves"].get(u, 0) for r in rec)]
    A = np.array([[r["waves"].get(u, 0) for u in units] for r in rec], float)
    c0 = np.array([UNIT_COST_SOURCE[u] for u in units], float)
    # relative residuals, the bench configs weighted 10x
    isb = np.array([r["scene"] in bench for r in rec])
    wgt = np.where(isb, 10.0, 1.0)
    c = solve(A, y, wgt, c0, lam)
    before, after = A @ c0 / y, A @ c / y
    # held-out figures: each bench config left out of its own fit, and a fit
    # without any bench config (the seeded scenes only)
    loo = {}
    for k, r in enumerate(rec):
        if r["scene"] in bench:
            keep = np.arange(len(rec)) != k
            ck = solve(A[keep], y[keep], wgt[keep], c0, lam)
            loo[r["scene"]] = float(A[k] @ ck / y[k])
    cn = solve(A[~isb], y[~isb], wgt[~isb], c0, lam)
    nob = {r["scene"]: float(A[k] @ cn / y[k]) for k, r in enumerate(rec) if r["scene"] in bench}
    print(f"{'scene':8s} {'PMC VALU':>12s} {'source/PMC':>11s} {'fitted':>8s} {'held out':>9s}")
    for k, (r, yy, b0, a0) in enumerate(zip(rec, y, before, after)):
        ho = f"{loo[r['scene']]:9.4f}" if r["scene"] in loo else ""
        print(f"{r['scene']:8s} {yy:12.4g} {b0:11.4f} {a0:8.4f} {ho}")
    print(f"rms rel. error: source prices {np.sqrt(np.mean((before - 1) ** 2)):.4f}, "
          f"fitted (in sample) {np.sqrt(np.mean((after - 1) ** 2)):.4f}")
    print("held out, each bench config left out of its own fit: " +
          ", ".join(f"{k} {v:.4f}" for k, v in loo.items()))
    print("held out, fit without any bench config: " +
          ", ".join(f"{k} {v:.4f}" for k, v in nob.items()))
    print("unit costs (source price -> fitted, bounds 0.6-1.7x the source price):")
    out = {}
    for u, a, b2 in zip(units, c0, c):
        out[u] = round(float(b2), 2)
        print(f"  {u:14s} {a:6.1f} -> {b2:7.2f}")
    json.dump({"lambda": lam, "costs": out, "prior": "UNIT_COST_SOURCE",
               "rms_before": float(np.sqrt(np.mean((before - 1) ** 2))),
               "rms_after": float(np.sqrt(np.mean((after - 1) ** 2))),
               "held_out_leave_one_config": loo, "held_out_no_bench_configs": nob},
              open(os.path.join(d, "fit.json"), "w"), indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--collect", default=None)
    ap.add_argument("--fit", default=None)
    ap.add_argument("--lam", type=float, default=0.02)
    a = ap.parse_args()
    if a.collect:
        collect(a.collect)
    if a.fit:
        fit(a.fit, a.lam)


if __name__ == "__main__":
    main()
