#!/usr/bin/env python3
"""tools/hostsim_counts.py [CONFIG] [ROW_STRIDE] — operation counts of the kernel
traversal (rtg_trace.h kCnt* slots, single-lane host build tests/hostsim) over a
row sample of a golden config, per primary sample and per LIVE sample (a sample
whose pixel is not +0, i.e. some ray of it reached a sphere).  Diagnostic only."""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import BUILD, GOLDEN, P, load_scene  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
from rtg_amd import UNIT_NAMES as NAMES  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    stride = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    hs = ctypes.CDLL(os.path.join(BUILD, "libhostsim.so"))
    c = json.load(open(os.path.join(GOLDEN, "golden.json")))["configs"][name]
    sph, lg = load_scene(name, c["spheres"], c["lights"])
    W, H, S = c["W"], c["H"], c["stack_size"]
    rows = np.arange(0, H, stride, dtype=np.uint32)
    out = np.zeros((len(rows), W, 3), np.float32)
    cnt = (ctypes.c_long * len(NAMES))()
    hs.hostsim_set_variant(0)
    hs.hostsim_counts(cnt, 1)
    rc = hs.hostsim_render_rows(P(sph), len(sph), P(lg), len(lg), W, H, ctypes.c_float(-4.0),
                                ctypes.c_float(3.0), S, P(rows), len(rows), P(out))
    assert rc == 0
    hs.hostsim_counts(cnt, 0)
    live_px = int(np.count_nonzero(np.any(out != 0, axis=2)))
    spp = cnt[0] / (len(rows) * W)
    live = live_px * spp
    print(f"{name}: {len(rows)} rows, {cnt[0]} samples, live pixels {live_px / (len(rows) * W):.3f}")
    for k, nm in enumerate(NAMES):
        print(f"  {nm:15s} {cnt[k]:14d}  /sample {cnt[k] / cnt[0]:8.3f}  /live {cnt[k] / live:8.3f}")


if __name__ == "__main__":
    main()
