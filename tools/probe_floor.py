"""tools/probe_floor.py — cost floor of the default kernel: C3-sized frames of
a scene whose spheres no primary ray reaches (every sample misses at once),
against the C3 scene itself.  Kernel time from HIP events, 20 launches."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
import rtg_amd as R  # noqa: E402


def time_scene(sph, lg, W=3840, H=2160, S=6, n=20, variant=0):
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    if variant:
        ctx.set_variant(variant)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    for _ in range(3):
        ctx.render_device(W, H, out.data_ptr(), stack_size=S, row_block=8, stream=s.cuda_stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        ctx.render_device(W, H, out.data_ptr(), stack_size=S, row_block=8, stream=s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    ctx.close()
    return e0.elapsed_time(e1) / n


variants = [int(v) for v in sys.argv[1:]] or [0]
sph, lg = R.generate_scene(16, 3, 42)
far = sph.copy()
far["pos"][:, 2] = 50.0  # behind the camera: every primary ray misses
for v in variants:
    print("variant %3d: c3 scene %.3f ms, all-miss (16 spheres) %.3f ms, no spheres %.3f ms" % (
        v, time_scene(sph, lg, variant=v), time_scene(far, lg, variant=v),
        time_scene(sph[:0], lg, variant=v)))
