#!/usr/bin/env python3
"""tools/chunk_rehearsal.py — one rank's part of bench.py's N > 1 step,
rehearsed on ONE GPU: rank 0's row-cyclic shard of G ranks rendered in K
chunks of whole row blocks on two streams in turn (render_rows_device, the
rows' global indices), exactly as bench.py issues them, after warm-up steps
(which give every chunk geometry its launch-order feedback).  Prints, per
(G, K), the mean render time of the shard and the predicted step

    T = render + the last chunk's gather (its bytes from each peer over one
        xGMI link at ~100 GB/s) + the last chunk's row-order restore (~5 TB/s)

so the chunk count can be chosen per config (more chunks overlap more of the
gather, but every launch ends with a tail of long waves).

  python tools/chunk_rehearsal.py --config c3 --ranks 2,4,8 --chunks 1,2,4
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))

CONFIGS = {"c2": (1920, 1080, 8, 2, 3), "c3": (3840, 2160, 16, 3, 5),
           "c4": (7680, 4320, 32, 4, 5), "c5": (3840, 2160, 1024, 4, 7)}
LINK_GBS = 100.0
ASSEMBLE_GBS = 5000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--ranks", default="2,4,8")
    ap.add_argument("--chunks", default="1,2,4")
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--last-frac", type=float, default=0.0,
                    help="the last chunk's share of the shard (0: equal chunks)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    import numpy as np
    import torch
    import rtg_amd as R
    from rtg_amd import dist as rdist
    W, H, n, m, depth = CONFIGS[a.config]
    S, B = depth + 1, a.row_block
    sph, lg = R.generate_scene(n, m, 42)
    torch.cuda.set_device(0)
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    main_s = torch.cuda.current_stream()
    rstreams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    out = []
    for G in [int(x) for x in a.ranks.split(",")]:
        Rmax = rdist.padded_rows(H, B, G)
        my_rows = R.shard_rows(H, B, 0, G)
        grow = torch.tensor(R.shard_row_indices(H, B, 0, G).astype(np.int64), dtype=torch.int32,
                            device="cuda")
        shard = torch.zeros((Rmax, W, 3), dtype=torch.float32, device="cuda")
        nblk = Rmax // B
        for K in [int(x) for x in a.chunks.split(",")]:
            K = max(1, min(K, nblk))
            bounds = rdist.chunk_bounds(nblk, K, B, a.last_frac)

            def step():
                for rs in rstreams:
                    rs.wait_stream(main_s)
                for c in range(K):
                    r0, r1 = bounds[c], bounds[c + 1]
                    nreal = max(0, min(r1, my_rows) - r0)
                    rs = rstreams[c % 2]
                    if nreal > 0:
                        ctx.render_rows_device(W, H, grow.data_ptr() + 4 * r0, nreal,
                                               shard.data_ptr() + 12 * W * r0, stack_size=S,
                                               stream=rs.cuda_stream)
                for rs in rstreams:
                    main_s.wait_stream(rs)

            for _ in range(3):
                step()
            torch.cuda.synchronize()
            ev[0].record(main_s)
            for _ in range(a.steps):
                step()
            ev[1].record(main_s)
            torch.cuda.synchronize()
            render = ev[0].elapsed_time(ev[1]) / a.steps
            last_rows = bounds[K] - bounds[K - 1]
            gather = last_rows * W * 12 / (LINK_GBS * 1e9) * 1e3 if G > 1 else 0.0
            assemble = 2 * last_rows * G * W * 12 / (ASSEMBLE_GBS * 1e9) * 1e3 if G > 1 else 0.0
            rec = {"config": a.config, "G": G, "K": K, "last_frac": a.last_frac, "bounds": bounds,
                   "render_ms": round(render, 4),
                   "last_gather_ms_est": round(gather, 4),
                   "last_assemble_ms_est": round(assemble, 4),
                   "predicted_step_ms": round(render + gather + assemble, 4)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
    ctx.close()
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
