#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the survey/build container only (needs /root/reference, via the
oracle/_ref/librtgref_S*.so libraries that oracle/build_ref.sh compiles from
it).  Outputs are data only — scene records, float32 framebuffers, hashes:

  golden.json            per-config metadata + hashes of full-size frames
  <name>.scene.bin       sphere records (n x 48 B) then light records (m x 24 B)
  <name>.small.f32       a small render of that scene (see golden.json)
  <name>.rows.f32        sampled full-width rows of the full-size frame
  case_<k>.scene.bin/.f32  seeded random edge-case scenes (empty scene,
                           no lights, S = 1, aa = 2.5, 1x1 frames, ...)

Float framebuffers are the reference's output bit for bit.  Hashes are taken
over canonical bits (every NaN as 0xFFC00000, see canon()).  Ray-sphere test counts come from the C
restatement (oracle/rtg_oracle.c), which is asserted bit-exact to the reference
on every frame generated here; the reference itself has no counters.

Usage: python tests/golden/make_golden.py [--quick]
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
import rtg_amd as R  # noqa: E402  (scene generator / PPM writer under test)

OUT = os.path.dirname(os.path.abspath(__file__))
NTHREADS = os.cpu_count() or 8

# (name, W, H, spheres, lights, depth, note) — BASELINE.json configs + the
# reference's own hard-coded scene.
CONFIGS = [
    ("ref800", 800, 600, 3, 2, 5, "main.cpp:104-168 scene as shipped (RTSTACK_MAXSIZE 6)"),
    ("c1", 640, 480, 4, 1, 1, "BASELINE configs[0]"),
    ("c2", 1920, 1080, 8, 2, 3, "BASELINE configs[1]"),
    ("c3", 3840, 2160, 16, 3, 5, "BASELINE configs[2] (bench workload)"),
    ("c4", 7680, 4320, 32, 4, 5, "BASELINE configs[3]"),
    ("c5", 3840, 2160, 1024, 4, 7, "BASELINE configs[4] (rows sampled only)"),
]
SMALL = (96, 54)


def P(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else None


def ref_lib(S):
    return ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", f"librtgref_S{S}.so"))


ORC = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "librtg_oracle.so"))


def ref_render(sph, lg, W, H, S, rows=None, aa=3.0, zoom=-4.0):
    rows = np.arange(H, dtype=np.uint32) if rows is None else np.asarray(rows, np.uint32)
    out = np.zeros((len(rows), W, 3), np.float32)
    ref_lib(S).ref_render_rows(P(sph), len(sph), P(lg), len(lg), W, H, ctypes.c_float(zoom),
                               ctypes.c_float(aa), P(rows), len(rows), P(out), NTHREADS)
    return out


def oracle_render(sph, lg, W, H, S, rows=None, aa=3.0, zoom=-4.0):
    rows = np.arange(H, dtype=np.uint32) if rows is None else np.asarray(rows, np.uint32)
    out = np.zeros((len(rows), W, 3), np.float32)
    cnt = (ctypes.c_ulonglong * 3)()
    ORC.oracle_render_rows(P(sph), len(sph), P(lg), len(lg), W, H, ctypes.c_float(zoom),
                           ctypes.c_float(aa), S, P(rows), len(rows), P(out), NTHREADS, cnt)
    return out, [int(c) for c in cnt]


def md5(b):
    return hashlib.md5(b).hexdigest()


def canon(fb):
    """uint32 bits with every NaN as 0xFFC00000.  IEEE-754 leaves NaN payloads
    (and signs) to the implementation: two x86 compilers of the same reference
    source already disagree on the sign of some NaNs (c4), so parity is
    bit-exact on every non-NaN value plus identical NaN positions."""
    b = np.ascontiguousarray(fb, np.float32).view(np.uint32).copy()
    b[np.isnan(fb)] = 0xFFC00000
    return b


def same(a, b):
    return a.shape == b.shape and bool((canon(a) == canon(b)).all())


def write_scene(name, sph, lg):
    with open(os.path.join(OUT, f"{name}.scene.bin"), "wb") as f:
        f.write(sph.tobytes())
        f.write(lg.tobytes())


def frame_meta(fb):
    bits = fb.view(np.uint32)
    nan = np.isnan(fb)
    pats = sorted({int(x) for x in np.unique(bits[nan])}) if nan.any() else []
    mx = R.max_colour_value(fb)
    return {"fb_md5": md5(canon(fb).tobytes()), "fb_md5_raw": md5(fb.tobytes()), "ppm_md5": md5(R.ppm_file_bytes(fb, mx)),
            "max_colour": float(np.float32(mx)), "max_colour_bits": int(np.float32(mx).view(np.uint32)),
            "nan_values": int(nan.sum()), "nan_patterns": [hex(p) for p in pats],
            "nonzero_px": int((fb.reshape(-1, 3) != 0).any(axis=1).sum())}


def sample_rows(H, k):
    rows = sorted({0, H - 1, H // 2, H // 2 - 1} | {int(r) for r in np.linspace(0, H - 1, k)})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true", help="skip c4 full frame and c5")
    args = ap.parse_args()
    meta = {"generator": "tests/golden/make_golden.py", "reference": "snowzurfer/raytracer-gamma "
            "raytracer.h via oracle/build_ref.sh", "seed": 42, "zoom": -4.0, "aliasFactor": 3.0,
            "small_size": list(SMALL), "configs": {}, "cases": []}
    for name, W, H, n, m, depth, note in CONFIGS:
        S = depth + 1
        sph, lg = R.generate_scene(n, m, 42)
        write_scene(name, sph, lg)
        c = {"W": W, "H": H, "spheres": n, "lights": m, "depth": depth, "stack_size": S,
             "note": note, "scene_md5": md5(sph.tobytes() + lg.tobytes())}
        t0 = time.time()
        # small render
        sw, sh = SMALL
        small = ref_render(sph, lg, sw, sh, S)
        o, _ = oracle_render(sph, lg, sw, sh, S)
        assert same(o, small), f"{name}: oracle != reference (small)"
        small.tofile(os.path.join(OUT, f"{name}.small.f32"))
        c["small"] = {"W": sw, "H": sh, "md5": md5(canon(small).tobytes())}
        if name == "c5" or (args.quick and name == "c4"):
            rows = [0, 270, 1079, 1080, 2159] if name == "c5" else sample_rows(H, 6)
            fb = ref_render(sph, lg, W, H, S, rows)
            o, cnt = oracle_render(sph, lg, W, H, S, rows)
            assert same(o, fb), f"{name}: oracle != ref rows"
            fb.tofile(os.path.join(OUT, f"{name}.rows.f32"))
            c["rows"] = {"rows": rows, "md5": md5(canon(fb).tobytes()), "ray_sphere_tests": cnt[0],
                         "nodes": cnt[1], "contain_tests": cnt[2]}
        else:
            fb = ref_render(sph, lg, W, H, S)
            o, cnt = oracle_render(sph, lg, W, H, S)
            assert same(o, fb), f"{name}: oracle != reference"
            c.update(frame_meta(fb))
            c["ray_sphere_tests"] = cnt[0]
            c["nodes"] = cnt[1]
            c["contain_tests"] = cnt[2]
            rows = sample_rows(H, 4)
            fb[rows].tofile(os.path.join(OUT, f"{name}.rows.f32"))
            c["rows"] = {"rows": rows, "md5": md5(canon(fb[rows]).tobytes())}
        c["gen_seconds"] = round(time.time() - t0, 1)
        meta["configs"][name] = c
        print(name, json.dumps({k: v for k, v in c.items() if k != "note"}), flush=True)

    # seeded edge cases
    rng = np.random.default_rng(20261015)
    spec = [  # (n, m, W, H, S, aa, zoom)
        (0, 2, 17, 9, 6, 3.0, -4.0),      # empty scene -> black
        (5, 0, 23, 13, 6, 3.0, -4.0),     # no lights -> matte 0
        (6, 2, 31, 17, 1, 3.0, -4.0),     # S = 1: root is a leaf
        (6, 2, 29, 11, 2, 2.5, -4.0),     # fractional aliasFactor (3x3 loop, 1/6.25)
        (6, 2, 1, 1, 6, 3.0, -4.0),       # 1x1 frame
        (7, 3, 40, 1, 6, 1.0, -2.0),      # single row, 1 spp, other zoom
        (9, 3, 1, 33, 9, 3.0, -6.0),      # single column, deep stack
        (12, 3, 37, 21, 12, 2.0, -4.0),   # ragged tiles, S = 12
        (10, 2, 45, 27, 4, 3.0, -4.0),
        (16, 4, 33, 19, 16, 3.0, -4.0),   # largest stack
    ]
    for k, (n, m, W, H, S, aa, zoom) in enumerate(spec):
        sph = np.zeros(n, R.SPHERE_DTYPE)
        for i in range(n):
            sph[i]["pos"] = [rng.uniform(-10, 10), rng.uniform(-7, 7), rng.uniform(-30, -3)]
            sph[i]["radius"] = rng.uniform(0.5, 4.0)
            sph[i]["material"] = R.make_material(
                float(rng.choice([0.0, 0.3, 0.6, 0.8, 1.0])), float(rng.uniform(0, 1)),
                rng.uniform(0, 1, 3), rng.uniform(0, 1, 3),
                float(rng.choice([1.0, 1.33, 1.55, 2.4])))
        lg = np.zeros(m, R.LIGHT_DTYPE)
        for l in range(m):
            lg[l]["pos"] = [rng.uniform(-60, 60), rng.uniform(-20, 80), rng.uniform(-40, 90)]
            lg[l]["col"] = rng.uniform(0.2, 1.0, 3)
        if S <= 16:
            fb = ref_render(sph, lg, W, H, S, aa=aa, zoom=zoom)
            src = "reference"
        else:  # beyond build_ref.sh's S range: the pinned restatement
            fb = None
            src = "restatement"
        o, cnt = oracle_render(sph, lg, W, H, S, aa=aa, zoom=zoom)
        if fb is not None:
            assert same(o, fb), f"case {k}: oracle != ref"
        else:
            fb = o
        name = f"case_{k}"
        write_scene(name, sph, lg)
        fb.tofile(os.path.join(OUT, f"{name}.f32"))
        meta["cases"].append({"name": name, "spheres": n, "lights": m, "W": W, "H": H,
                              "stack_size": S, "aliasFactor": aa, "zoom": zoom,
                              "source": src, "md5": md5(canon(fb).tobytes()),
                              "ray_sphere_tests": cnt[0]})
        print(name, n, m, W, H, S, aa, zoom, src, flush=True)
    with open(os.path.join(OUT, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote", os.path.join(OUT, "golden.json"))


if __name__ == "__main__":
    main()
