#!/usr/bin/env python3
"""tools/time_semantics.py [CONFIG] [ROUNDS] — interleaved kernel times of the
CPU-semantics default kernel and the OpenCL-semantics one (f32 Fresnel and
sinA1, otherwise nearly the same work): an upper bound on what the f64 islands
of calculateRefraction cost.  Diagnostic only (GPU)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
sys.path.insert(0, ROOT)
import rtg_amd as R  # noqa: E402
from bench import CONFIGS  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c3"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    W, H, n, m, depth = CONFIGS[name]
    sph, lg = R.generate_scene(n, m, 42)
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = {"cpu": [], "opencl": []}
    for _ in range(rounds):
        for sem, key in ((R.Context.SEMANTICS_CPU, "cpu"), (R.Context.SEMANTICS_OPENCL, "opencl")):
            ctx.set_semantics(sem)
            S = depth + 1  # same stack size for both: same tree depth
            ctx.render_device(W, H, out.data_ptr(), stack_size=S, stream=s.cuda_stream)
            e0.record(s)
            for _ in range(5):
                ctx.render_device(W, H, out.data_ptr(), stack_size=S, stream=s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            times[key].append(e0.elapsed_time(e1) / 5)
    print(name, {k: round(float(np.median(v)), 4) for k, v in times.items()}, flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
