#!/usr/bin/env python3
"""Cold-launch probe: after the GPU is warm, time the
first launches of a fresh frame geometry one by one (set_scene bumps the
scene generation, so the launch-order feedback starts empty), with the
feedback on and off, and back-to-back steady launches for reference.

  python tools/cold_probe.py --config c3 [--reps 3] [--json out.json]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import torch
    import rtg_amd as R
    from bench import CONFIGS
    W, H, n, m, depth = CONFIGS[a.config]
    S = depth + 1
    sph, lg = R.generate_scene(n, m)
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    fb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def one():
        e0.record(st)
        ctx.render_device(W, H, fb.data_ptr(), stack_size=S, stream=st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    for _ in range(20):  # warm the GPU (clocks, code objects, launch scratch)
        one()
    out = {"config": a.config}
    for name, flags in (("feedback", 0), ("no_feedback", ctx.LAUNCH_NO_ORDER_FEEDBACK)):
        ctx.set_variant(0, flags)
        seqs = []
        for _ in range(a.reps):
            ctx.set_scene(sph, lg)  # new scene generation: no feedback yet
            torch.cuda.synchronize()
            seqs.append([one() for _ in range(a.launches)])
        steady = []
        for _ in range(10):
            steady.append(one())
        out[name] = {"per_launch_ms": seqs, "steady_ms": float(np.median(steady))}
        print(a.config, name, "launch k of a fresh geometry (ms):",
              " | ".join(" ".join(f"{t:.3f}" for t in s) for s in seqs),
              f"; steady {np.median(steady):.3f}", flush=True)
    ctx.set_variant(0, 0)
    ctx.close()
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
