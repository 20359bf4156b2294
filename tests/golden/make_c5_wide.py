#!/usr/bin/env python3
"""Widened C5 fixture (3840x2160, 1024 spheres, 4 lights, depth 7) from the
REFERENCE itself (oracle/_ref/librtgref_S8.so, built from raytracer.h by
oracle/build_ref.sh).  A whole C5 frame costs days of CPU in the reference, so
the fixture is a sample:

  * every 32nd full-width row, the 16 rows of the centre band (1072..1087,
    the costliest rows: most rays enter the sphere cluster there) and the
    last row;
  * 100,000 pixels drawn uniformly from the whole frame (seeded).

Output: tests/golden/c5.wide.npz (compressed; data only: row indices, pixel
ids and the reference's float32 values) and a "wide" entry under
golden.json's c5 config with the canonical-bits md5s.  A few rows are also
rendered by the C restatement (oracle/rtg_oracle.c) and asserted bit-exact.

Run in the build container only (needs /root/reference via oracle/_ref):
  python tests/golden/make_c5_wide.py
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
import rtg_amd as R  # noqa: E402  (scene generator)

OUT = os.path.dirname(os.path.abspath(__file__))
NTHREADS = os.cpu_count() or 8
W, H, NS, NL, S = 3840, 2160, 1024, 4, 8
NPIX = 100_000


def P(a):
    return ctypes.c_void_p(a.ctypes.data) if a.size else None


def canon(fb):
    b = np.ascontiguousarray(fb, np.float32).view(np.uint32).copy()
    b[np.isnan(fb)] = 0xFFC00000
    return b


def wide_rows():
    return sorted(set(range(0, H, 32)) | set(range(H // 2 - 8, H // 2 + 8)) | {H - 1})


def main():
    ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", f"librtgref_S{S}.so"))
    orc = ctypes.CDLL(os.path.join(ROOT, "oracle", "build", "librtg_oracle.so"))
    sph, lg = R.generate_scene(NS, NL, 42)
    raw = open(os.path.join(OUT, "c5.scene.bin"), "rb").read()
    assert raw == sph.tobytes() + lg.tobytes(), "c5.scene.bin is not the seed-42 scene"
    rows = np.asarray(wide_rows(), np.uint32)
    t0 = time.time()
    fb = np.zeros((len(rows), W, 3), np.float32)
    ref.ref_render_rows(P(sph), NS, P(lg), NL, W, H, ctypes.c_float(-4.0), ctypes.c_float(3.0),
                        P(rows), len(rows), P(fb), NTHREADS)
    t_rows = time.time() - t0
    print(f"{len(rows)} rows in {t_rows:.1f} s", flush=True)
    rng = np.random.default_rng(20261017)
    gids = np.sort(rng.choice(W * H, size=NPIX, replace=False)).astype(np.uint32)
    t0 = time.time()
    px = np.zeros((NPIX, 3), np.float32)
    ref.ref_render_pixels(P(sph), NS, P(lg), NL, W, H, ctypes.c_float(-4.0),
                          ctypes.c_float(3.0), P(gids), NPIX, P(px), NTHREADS)
    t_px = time.time() - t0
    print(f"{NPIX} pixels in {t_px:.1f} s", flush=True)
    # the C restatement agrees on a few rows (centre band included)
    chk = np.asarray([0, 1080, 1084, 1600], np.uint32)
    o = np.zeros((len(chk), W, 3), np.float32)
    cnt = (ctypes.c_ulonglong * 3)()
    orc.oracle_render_rows(P(sph), NS, P(lg), NL, W, H, ctypes.c_float(-4.0), ctypes.c_float(3.0),
                           S, P(chk), len(chk), P(o), NTHREADS, cnt)
    idx = [int(np.searchsorted(rows, r)) for r in chk]
    assert (canon(o) == canon(fb[idx])).all(), "oracle != reference on the check rows"
    np.savez_compressed(os.path.join(OUT, "c5.wide.npz"), rows=rows, rows_fb=fb, gids=gids,
                        pixels=px)
    gj = os.path.join(OUT, "golden.json")
    meta = json.load(open(gj))
    meta["configs"]["c5"]["wide"] = {
        "file": "c5.wide.npz", "rows": len(rows), "pixels": NPIX, "pixel_seed": 20261017,
        "rows_md5": hashlib.md5(canon(fb).tobytes()).hexdigest(),
        "pixels_md5": hashlib.md5(canon(px).tobytes()).hexdigest(),
        "nan_values": int(np.isnan(fb).sum() + np.isnan(px).sum()),
        "nonzero_px": int((fb.reshape(-1, 3) != 0).any(axis=1).sum() + (px != 0).any(axis=1).sum()),
        "gen_seconds": round(t_rows + t_px, 1), "threads": NTHREADS,
        "generator": "tests/golden/make_c5_wide.py"}
    with open(gj, "w") as f:
        json.dump(meta, f, indent=1)
    print("wrote c5.wide.npz", meta["configs"]["c5"]["wide"])


if __name__ == "__main__":
    main()
