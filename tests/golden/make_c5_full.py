#!/usr/bin/env python3
"""Whole-frame C5 pin (3840x2160, 1024 spheres, 4 lights, depth 7) from the
REFERENCE itself (oracle/_ref/librtgref_S8.so, built from raytracer.h by
oracle/build_ref.sh), plus the C restatement's ray-sphere test counts.

The frame costs the reference ~2 h on the 8-core build container, so it is
rendered in row chunks that are kept under tests/_build/c5_full/ (git- and
gpurun-ignored) and the run resumes where it stopped:

  stage 1  reference rows  -> ref_<k>.npy            (the pinned frame)
  stage 2  restatement rows + counters -> cnt_<k>.json, asserted bit-exact
           to the reference chunk (a whole-frame check of the oracle)

At the end the canonical-bits frame md5, the raw md5, NaN count, the max
colour (maxColourValuePixelBuffer, algebra.h:68-91, called in the reference
build) and the PPM md5 (savePPM semantics, main.cpp:43-91, via
rtg_amd.ppm_file_bytes) go into golden.json's c5 entry, next to the counters.
Data only; no reference source is stored.

Run in the build container only:  nice -n 19 python tests/golden/make_c5_full.py
"""
from __future__ import annotations

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
WORK = os.path.join(ROOT, "tests", "_build", "c5_full")
NTHREADS = int(os.environ.get("C5_THREADS", os.cpu_count() or 8))
W, H, NS, NL, S = 3840, 2160, 1024, 4, 8
CHUNK = 40  # rows per chunk (54 chunks)


def P(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else None


def canon(fb):
    b = np.ascontiguousarray(fb, np.float32).view(np.uint32).copy()
    b[np.isnan(fb)] = 0xFFC00000
    return b


def main():
    os.makedirs(WORK, exist_ok=True)
    ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", f"librtgref_S{S}.so"))
    orc = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "librtg_oracle.so"))
    ref.ref_max_colour.restype = ctypes.c_float
    sph, lg = R.generate_scene(NS, NL, 42)
    raw = open(os.path.join(OUT, "c5.scene.bin"), "rb").read()
    assert raw == sph.tobytes() + lg.tobytes(), "c5.scene.bin is not the seed-42 scene"
    nck = (H + CHUNK - 1) // CHUNK
    args = (P(sph), NS, P(lg), NL, W, H, ctypes.c_float(-4.0), ctypes.c_float(3.0))
    for stage in ("ref", "cnt"):
        for k in range(nck):
            rows = np.arange(k * CHUNK, min(H, (k + 1) * CHUNK), dtype=np.uint32)
            f_ref = os.path.join(WORK, f"ref_{k:03d}.npy")
            f_cnt = os.path.join(WORK, f"cnt_{k:03d}.json")
            if stage == "ref" and os.path.exists(f_ref):
                continue
            if stage == "cnt" and os.path.exists(f_cnt):
                continue
            t0 = time.time()
            fb = np.zeros((len(rows), W, 3), np.float32)
            if stage == "ref":
                ref.ref_render_rows(*args, P(rows), len(rows), P(fb), NTHREADS)
                np.save(f_ref + ".tmp.npy", fb)
                os.replace(f_ref + ".tmp.npy", f_ref)
            else:
                cnt = (ctypes.c_ulonglong * 3)()
                orc.oracle_render_rows(*args, S, P(rows), len(rows), P(fb), NTHREADS, cnt)
                want = np.load(f_ref)
                assert (canon(fb) == canon(want)).all(), f"oracle != reference in chunk {k}"
                with open(f_cnt, "w") as f:
                    json.dump({"rows": [int(rows[0]), int(rows[-1])], "counts": [int(c) for c in cnt],
                               "seconds": round(time.time() - t0, 1)}, f)
            print(f"{stage} chunk {k + 1}/{nck} rows {rows[0]}-{rows[-1]} "
                  f"{time.time() - t0:.1f} s", flush=True)
    fb = np.concatenate([np.load(os.path.join(WORK, f"ref_{k:03d}.npy")) for k in range(nck)])
    assert fb.shape == (H, W, 3)
    cnts = [json.load(open(os.path.join(WORK, f"cnt_{k:03d}.json"))) for k in range(nck)]
    tot = [sum(c["counts"][i] for c in cnts) for i in range(3)]
    mx = ref.ref_max_colour(P(fb), ctypes.c_ulonglong(W * H))
    assert np.float32(mx) == np.float32(R.max_colour_value(fb)), "max colour: harness != rtg_amd"
    nan = np.isnan(fb)
    bits = fb.view(np.uint32)
    wide = np.load(os.path.join(OUT, "c5.wide.npz"))
    assert (canon(fb[wide["rows"]]) == canon(wide["rows_fb"])).all(), "full frame != wide rows"
    assert (canon(fb.reshape(-1, 3)[wide["gids"]]) == canon(wide["pixels"])).all(), \
        "full frame != wide pixels"
    full = {
        "fb_md5": hashlib.md5(canon(fb).tobytes()).hexdigest(),
        "fb_md5_raw": hashlib.md5(fb.tobytes()).hexdigest(),
        "ppm_md5": hashlib.md5(R.ppm_file_bytes(fb, mx)).hexdigest(),
        "max_colour": float(np.float32(mx)),
        "max_colour_bits": int(np.float32(mx).view(np.uint32)),
        "nan_values": int(nan.sum()),
        "nan_patterns": [hex(p) for p in sorted({int(x) for x in np.unique(bits[nan])})],
        "nonzero_px": int((fb.reshape(-1, 3) != 0).any(axis=1).sum()),
        "ray_sphere_tests": tot[0], "nodes": tot[1], "contain_tests": tot[2],
        "generator": "tests/golden/make_c5_full.py", "threads": NTHREADS,
        "chunks": nck,
    }
    gj = os.path.join(OUT, "golden.json")
    meta = json.load(open(gj))
    c5 = meta["configs"]["c5"]
    c5.update(full)
    c5["note"] = "BASELINE configs[4] (whole frame pinned by make_c5_full.py)"
    with open(gj, "w") as f:
        json.dump(meta, f, indent=1)
    print("c5 full:", json.dumps(full))


if __name__ == "__main__":
    main()
