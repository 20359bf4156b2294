#!/usr/bin/env python3
"""tools/order_ab.py — launch-order A/B on one GPU: the full frame and the
eight 1/8 row-cyclic shards (B = 8, each rendered alone, as one rank of an
8-GPU frame renders it) of a config, timed with HIP events after warm-up
renders (which give the launch-order feedback its measured group times).
The library comes from RTG_LIB, the order from RTG_LAUNCH_ORDER (unset:
feedback; "popcount": the sphere-count order).  Prints one JSON line:
full-frame ms, per-shard ms (median of R), the largest shard, their sum and
whether the frame and the assembled shards match the golden md5.

  RTG_LIB=ab/librtg_x.so python tools/order_ab.py --config c3
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--shards", type=int, default=8)
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    import torch
    import rtg_amd as R
    from rtg_amd import dist
    from conftest import canon_md5, load_scene
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    c = g["configs"][a.config]
    sph, lg = load_scene(a.config, c["spheres"], c["lights"])
    W, H, S, B, G = c["W"], c["H"], c["stack_size"], a.row_block, a.shards
    torch.cuda.set_device(0)
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    st = torch.cuda.current_stream()
    sp = st.cuda_stream
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for _ in range(3):
        ctx.render_device(W, H, out.data_ptr(), stack_size=S, row_block=B, stream=sp)
    torch.cuda.synchronize()
    ev[0].record(st)
    for _ in range(a.steps):
        ctx.render_device(W, H, out.data_ptr(), stack_size=S, row_block=B, stream=sp)
    ev[1].record(st)
    torch.cuda.synchronize()
    full_ms = ev[0].elapsed_time(ev[1]) / a.steps
    full_ok = canon_md5(out.cpu().numpy()) == c.get("fb_md5")
    Rmax = dist.padded_rows(H, B, G)
    buf = torch.zeros((G, Rmax, W, 3), dtype=torch.float32, device="cuda")
    shard_ms = []
    for s in range(G):
        for _ in range(3):
            ctx.render_device(W, H, buf[s].data_ptr(), stack_size=S, row_block=B, shard=s,
                              n_shards=G, stream=sp)
        ts = []
        for _ in range(a.reps):
            ev[0].record(st)
            ctx.render_device(W, H, buf[s].data_ptr(), stack_size=S, row_block=B, shard=s,
                              n_shards=G, stream=sp)
            ev[1].record(st)
            torch.cuda.synchronize()
            ts.append(ev[0].elapsed_time(ev[1]))
        shard_ms.append(float(np.median(ts)))
    shards_ok = canon_md5(dist.assemble(buf, H, B).cpu().numpy()) == c.get("fb_md5")
    print(json.dumps({"config": a.config, "lib": os.path.basename(os.environ.get("RTG_LIB", "librtg.so")),
                      "order": os.environ.get("RTG_LAUNCH_ORDER", "feedback"),
                      "full_ms": round(full_ms, 4), "shard_ms": [round(x, 4) for x in shard_ms],
                      "shard_max_ms": round(max(shard_ms), 4), "shard_sum_ms": round(sum(shard_ms), 4),
                      "full_md5_ok": full_ok, "shards_md5_ok": shards_ok}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
