#!/usr/bin/env python3
"""Per-lane executed-work counts of the kernel traversal on the small golden
frames, from the host build of rtg_trace.h (tests/hostsim): the units whose
per-lane count is a fact of the algorithm (shading, lights, shadow rays,
refraction, reflection pushes, descents, unwind steps), independent of how
lanes share waves.  tests/test_gpu_parity.py checks the device counting build
(variant 120, lane-level counters) against them; tests/test_oracle.py checks
this fixture against the current hostsim.

  python tests/golden/make_unit_counts.py     -> tests/golden/unit_counts.json
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
import rtg_amd as R  # noqa: E402
from conftest import BUILD, P, load_scene  # noqa: E402

NAMES = ["ref800", "c2", "c3"]
UNITS = ["U.shade", "U.light", "U.shadow", "U.lit", "U.refr", "U.refrLeaf", "U.push",
         "U.descend", "U.unwind"]


def hostsim_counts(hs, golden):
    res = {}
    for name in NAMES:
        c = golden["configs"][name]
        sph, lg = load_scene(name, c["spheres"], c["lights"])
        W, H = c["small"]["W"], c["small"]["H"]
        rows = np.arange(H, dtype=np.uint32)
        out = np.zeros((H, W, 3), np.float32)
        cnt = (ctypes.c_long * len(R.UNIT_NAMES))()
        hs.hostsim_set_variant(0)
        hs.hostsim_counts(cnt, 1)
        rc = hs.hostsim_render_rows(P(sph), len(sph), P(lg), len(lg), W, H, ctypes.c_float(-4.0),
                                    ctypes.c_float(3.0), c["stack_size"], P(rows), H, P(out))
        assert rc == 0
        hs.hostsim_counts(cnt, 1)
        res[name] = {u: int(cnt[R.UNIT_NAMES.index(u)]) for u in UNITS}
    return res


def main():
    hs = ctypes.CDLL(os.path.join(BUILD, "libhostsim.so"))
    golden = json.load(open(os.path.join(HERE, "golden.json")))
    res = hostsim_counts(hs, golden)
    json.dump({"generator": "tests/golden/make_unit_counts.py", "units": UNITS, "frames": res},
              open(os.path.join(HERE, "unit_counts.json"), "w"), indent=1)
    print(res)


if __name__ == "__main__":
    main()
