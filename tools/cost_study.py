#!/usr/bin/env python3
"""Launch-order study (the cold launch).

GPU part (`--dump`): renders a bench config's frame a few times so that the
launch-order feedback has the groups' measured trace times, then saves the
last launch's cost table, list, sphere masks and run lengths
(rtg_diag_group_list) with the scene, plus the cold and fed frame times.

CPU part (`--analyse file.npz`): replays the measured group times through
greedy list scheduling on the trace kernel's resident wave slots (a wave per
listed group, taken in list order as slots free up) for candidate orders a
cull pass can compute without a previous launch, against the measured
(feedback) order.

  python tools/cost_study.py --dump --config c3 --out gpurun_out/cost_c3.npz
  python tools/cost_study.py --analyse gpurun_out/cost_c3.npz
"""
import argparse
import heapq
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
sys.path.insert(0, ROOT)


def dump(cfg, out, reps):
    import torch
    import rtg_amd as R
    from bench import CONFIGS
    W, H, n, m, depth = CONFIGS[cfg]
    S = depth + 1
    sph, lg = R.generate_scene(n, m)
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    fb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for _ in range(reps):
        e0.record(st)
        ctx.render_device(W, H, fb.data_ptr(), stack_size=S, stream=st.cuda_stream)
        e1.record(st)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    d = ctx.diag_group_list()
    np.savez_compressed(out, cost=d["cost"], list=d["list"], sel=d["sel"], runs=d["runs"],
                        times=np.array(times), W=W, H=H, sph=sph.view(np.uint8),
                        lg=lg.view(np.uint8), numcu=torch.cuda.get_device_properties(0)
                        .multi_processor_count)
    print(cfg, "frame ms per launch:", " ".join(f"{t:.3f}" for t in times))
    ctx.close()


def listed(d):
    """(group, sel) of every listed group, in the trace kernel's order."""
    n = int(d["runs"].sum())
    return d["list"][:n].astype(np.int64), d["sel"][:n]


def makespan(costs, slots):
    """Greedy list scheduling: each job to the first slot that frees."""
    h = [0.0] * slots
    for c in costs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + c)
    return max(h)


def analyse(path, slots):
    import rtg_amd as R
    d = dict(np.load(path))
    g, sel = listed(d)
    cost = d["cost"][g].astype(np.float64) / 100.0  # us
    sph = d["sph"].view(R.SPHERE_DTYPE)
    mat = sph["material"]
    n = len(sph)
    bits = ((sel[:, None] >> np.arange(n, dtype=np.uint64)[None, :]) & np.uint64(1)).astype(bool)
    pc = bits.sum(1)
    opac = mat["opacity"]
    gloss = mat["glossColour"].max(1)
    transp = (1.0 - opac) > 0
    print(f"{path}: {len(g)} listed groups, frame ms {d['times']}, slots {slots}")
    print(f"cost us: mean {cost.mean():.1f} p50 {np.median(cost):.1f} p99 "
          f"{np.percentile(cost, 99):.1f} max {cost.max():.1f}; sum/slots "
          f"{cost.sum() / slots:.1f} us")
    cands = {
        "feedback (measured, descending)": -cost,
        "list order as is": np.arange(len(g)),
        "popcount >= 2 first": -(pc >= 2).astype(float),
        "popcount": -pc.astype(float),
        "transparent spheres in mask": -(bits & transp[None, :]).sum(1).astype(float),
        "sum w (1 + 3 transp + gloss)": -(bits * (1 + 3 * transp + gloss)[None, :]).sum(1),
        "group index (image order)": g.astype(float),
    }
    rng = np.random.default_rng(0)
    cands["random"] = rng.permutation(len(g)).astype(float)
    for name, key in cands.items():
        order = np.argsort(key, kind="stable")
        ms = makespan(cost[order], slots)
        print(f"  {name:34s} makespan {ms:8.1f} us")
    # how well do features rank costs: mean cost per popcount / transparent count
    for k in range(0, min(n, 8) + 1):
        s = pc == k
        if s.any():
            print(f"  popcount {k}: {s.sum():7d} groups, mean cost {cost[s].mean():7.1f} us")
    tc = (bits & transp[None, :]).sum(1)
    for k in range(0, 6):
        s = tc == k
        if s.any():
            print(f"  transparent {k}: {s.sum():7d} groups, mean cost {cost[s].mean():7.1f} us")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dump", action="store_true")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--analyse", default=None)
    ap.add_argument("--slots", type=int, default=8192)
    a = ap.parse_args()
    if a.dump:
        dump(a.config, a.out or f"gpurun_out/cost_{a.config}.npz", a.reps)
    if a.analyse:
        analyse(a.analyse, a.slots)


if __name__ == "__main__":
    main()
