"""tools/probe_launch.py — host-side cost of one render call (ctypes + the C
ABI's launch path: cull pass, trace kernel, event), from 2000 back-to-back
renders of a 7 x 1 frame whose GPU work is negligible."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
import rtg_amd as R  # noqa: E402

sph, lg = R.generate_scene(16, 3, 42)
ctx = R.Context(0)
ctx.set_scene(sph, lg)
out = torch.empty((64, 64, 3), dtype=torch.float32, device="cuda")
rows = torch.arange(64, dtype=torch.int32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
for name, fn in [("render_device", lambda: ctx.render_device(7, 1, out.data_ptr(), stream=s)),
                 ("render_rows_device", lambda: ctx.render_rows_device(7, 1, rows.data_ptr(), 1,
                                                                       out.data_ptr(), stream=s))]:
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(2000):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name}: host {1e6 * (t1 - t0) / 2000:.1f} us/call, "
          f"with drain {1e6 * (t2 - t0) / 2000:.1f} us/call")
ctx.close()
