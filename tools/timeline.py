#!/usr/bin/env python3
"""Wave-occupancy timeline of the trace kernel (diagnostic, GPU box).

Renders a config with a kernel variant and the RTG_LAUNCH_TIMELINE flag (one
{start, end, HW_ID, XCC_ID} record per wave, s_memrealtime at 100 MHz) and
reports how full the SIMDs' wave slots were over the launch: mean resident
waves per SIMD, the occupancy curve over time, wave-duration spread, and the
slot time lost to workgroups waiting for their slowest wave.

  python tools/timeline.py [--config c3] [--json out.json]
"""
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
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--waves-per-block", type=int, default=4)
    ap.add_argument("--json", default=None)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--shards", type=int, default=1)
    ap.add_argument("--row-block", type=int, default=8)
    ap.add_argument("--raw", default=None, help="also save the per-wave records (t0, t1 in "
                    "10 ns ticks from the first start, hw id, xcc id; index = the wave's "
                    "list position) to this .npz")
    a = ap.parse_args()
    import torch
    import rtg_amd as R
    from conftest import load_scene
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    c = g["configs"][a.config]
    sph, lg = load_scene(a.config, c["spheres"], c["lights"])
    W, H, S = c["W"], c["H"], c["stack_size"]
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    ctx.set_variant(a.variant, ctx.LAUNCH_TIMELINE)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    for _ in range(3):
        ev[0].record()
        ctx.render_device(W, H, out.data_ptr(), stack_size=S, row_block=a.row_block,
                          shard=a.shard, n_shards=a.shards, stream=st)
        ev[1].record()
    torch.cuda.synchronize()
    rec = ctx.diag_timeline().astype(np.int64)
    t0 = rec[:, 0]
    t1 = rec[:, 1]
    t1 = np.where(t1 < t0, t1 + (1 << 32), t1)
    base = t0.min()
    t0 -= base
    t1 -= base
    span = t1.max()
    dur = t1 - t0
    hw, xcc = rec[:, 2], rec[:, 3] & 15
    tag = rec[:, 3] >> 4  # compacted launches: first group's mask popcount, group index
    if a.raw:
        np.savez_compressed(a.raw, t0=t0.astype(np.int32), t1=t1.astype(np.int32),
                            hw=hw.astype(np.uint32), xcc=xcc.astype(np.uint8),
                            popcount=(tag & 127).astype(np.uint8), group=(tag >> 7).astype(np.int32))
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    nsimd = len(np.unique(key))
    ncu = len(np.unique(key // 4))
    mean_res = dur.sum() / (span * nsimd)
    # occupancy curve: resident waves per SIMD at 40 instants
    ts = np.linspace(0, span, 41)[:-1] + span / 80
    curve = [float(((t0 <= t) & (t1 > t)).sum() / nsimd) for t in ts]
    wpb = a.waves_per_block
    nb = len(dur) // wpb
    blk = dur[:nb * wpb].reshape(nb, wpb)
    blk_end = t1[:nb * wpb].reshape(nb, wpb).max(1, keepdims=True)
    held_idle = (blk_end - t1[:nb * wpb].reshape(nb, wpb)).sum()
    # per-SIMD peak concurrency
    order = np.argsort(key, kind="stable")
    # the last 10 % of the span: resident waves per SIMD (the tail)
    tail = [float(((t0 <= t) & (t1 > t)).sum() / nsimd) for t in np.linspace(0.9 * span, span, 11)[:-1]]
    res = {
        "config": a.config, "variant": a.variant, "shard": [a.shard, a.shards, a.row_block],
        "launch_ms_events": float(ev[0].elapsed_time(ev[1])), "waves": int(len(dur)),
        "tail_last10pct_resident": [round(v, 2) for v in tail],
        "span_us": span / 100.0, "simds_seen": int(nsimd), "cus_seen": int(ncu),
        "mean_resident_waves_per_simd": float(mean_res),
        "occupancy_curve": [round(v, 2) for v in curve],
        "wave_us": {"mean": float(dur.mean() / 100), "p50": float(np.percentile(dur, 50) / 100),
                    "p90": float(np.percentile(dur, 90) / 100),
                    "p99": float(np.percentile(dur, 99) / 100), "max": float(dur.max() / 100)},
        "slot_time_held_by_finished_waves": float(held_idle / (span * nsimd)),
        "first_start_last_start_us": [0.0, float(t0.max() / 100)],
        "ramp_up_us_to_half": float(np.percentile(t0, 5) / 100),
    }
    print(json.dumps(res, indent=1))
    if a.json:
        json.dump(res, open(a.json, "w"), indent=1)
    ctx.close()


if __name__ == "__main__":
    main()
