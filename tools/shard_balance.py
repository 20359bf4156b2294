#!/usr/bin/env python3
"""tools/shard_balance.py — the multi-GPU row deal rehearsed on ONE GPU
(SURVEY.md §8e): for G = 1, 2, 4, 8 ranks and row blocks of B rows, render
each rank's row-cyclic shard (rtg_render_device, shard g of G) alone, timed
with HIP events (median of R repetitions), and count its executed work with
the counting build (variant 120, VALU slots priced by rtg_amd/work.py).

Per (G, B) it reports every shard's render ms and work, the imbalance
max/mean, and the predicted G-GPU frame time
    T_G = max_g t_g + gather tail + assemble
with the gather tail = the last of K = 4 pipelined chunks of the largest
shard over one xGMI link (the other chunks overlap rendering; 7 x 153 GB/s
links per GPU, ~100 GB/s of it sustained per peer) and the assemble = the last
chunk's read + write on the root at ~5 TB/s (bench.py restores each chunk's
row order on a third stream as it arrives, so the earlier chunks' restores
overlap rendering).  speedup_G = T_1 / T_G.

  python tools/shard_balance.py [--config c4] [--blocks 4,8,16] [--json OUT]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
import rtg_amd as R  # noqa: E402
from rtg_amd import dist as rdist  # noqa: E402
from rtg_amd import work as rwork  # noqa: E402

CONFIGS = {"c2": (1920, 1080, 8, 2, 3), "c3": (3840, 2160, 16, 3, 5),
           "c4": (7680, 4320, 32, 4, 5), "c5": (3840, 2160, 1024, 4, 7)}
LINK_GBS = 100.0     # sustained per-peer xGMI rate assumed for the gather tail
ASSEMBLE_GBS = 5000.0
CHUNKS = 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--blocks", default="4,8,16")
    ap.add_argument("--ranks", default="1,2,4,8")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    W, H, n, m, depth = CONFIGS[a.config]
    S = depth + 1
    sph, lg = R.generate_scene(n, m, 42)
    torch.cuda.set_device(0)
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    buf = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    for _ in range(2):  # warm-up
        ctx.render_device(W, H, buf.data_ptr(), stack_size=S, stream=sptr)
    torch.cuda.synchronize()

    def shard_run(g, G, B):
        ts = []
        for _ in range(2):  # warm-up: gives the launch-order feedback its group times
            ctx.render_device(W, H, buf.data_ptr(), stack_size=S, row_block=B, shard=g,
                              n_shards=G, stream=sptr)
        for _ in range(a.reps):
            e0.record(stream)
            ctx.render_device(W, H, buf.data_ptr(), stack_size=S, row_block=B, shard=g,
                              n_shards=G, stream=sptr)
            e1.record(stream)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ctx.set_variant(120)
        ctx.diag_counts(reset=True)
        ctx.render_device(W, H, buf.data_ptr(), stack_size=S, row_block=B, shard=g,
                          n_shards=G, stream=sptr)
        torch.cuda.synchronize()
        wv, _ = ctx.diag_counts(reset=True)
        ctx.set_variant(0)
        return float(np.median(ts)), int(rwork.executed_work(R.UNIT_NAMES, wv)["valu_slots"])

    t1, w1 = shard_run(0, 1, 8)
    out = {"config": a.config, "W": W, "H": H, "frame_ms_1gpu": round(t1, 4),
           "frame_valu_slots": w1, "assumptions": {
               "gather_tail": f"last of {CHUNKS} chunks of the largest shard over one link at "
                              f"{LINK_GBS} GB/s", "assemble": f"the last of {CHUNKS} chunks' read+write at {ASSEMBLE_GBS} GB/s"},
           "cases": []}
    for B in [int(x) for x in a.blocks.split(",")]:
        for G in [int(x) for x in a.ranks.split(",")]:
            ms, wk = [], []
            for g in range(G):
                t, w = shard_run(g, G, B)
                ms.append(round(t, 4))
                wk.append(w)
            Rmax = rdist.padded_rows(H, B, G)
            shard_bytes = Rmax * W * 12
            gather_tail = (shard_bytes / CHUNKS) / (LINK_GBS * 1e9) * 1e3 if G > 1 else 0.0
            assemble = (2 * W * H * 12 / CHUNKS) / (ASSEMBLE_GBS * 1e9) * 1e3 if G > 1 else 0.0
            tG = max(ms) + gather_tail + assemble
            case = {"G": G, "B": B, "shard_ms": ms, "shard_valu_slots": wk,
                    "imbalance_time": round(max(ms) / (sum(ms) / G), 4),
                    "imbalance_work": round(max(wk) / (sum(wk) / G), 4),
                    "gather_tail_ms_est": round(gather_tail, 4),
                    "assemble_ms_est": round(assemble, 4),
                    "predicted_frame_ms": round(tG, 4),
                    "predicted_speedup": round(t1 / tG, 3),
                    "render_speedup": round(t1 / max(ms), 3)}
            out["cases"].append(case)
            print(json.dumps(case), flush=True)
    ctx.close()
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()
