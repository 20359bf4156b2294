#!/usr/bin/env python3
"""bench.py — raytracer-gamma hot path on MI355X: Mpixels/s of the per-pixel
Whitted raytrace (librtg.so HIP kernel) on BASELINE.json's configs[2] workload.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3]
  torchrun --nproc-per-node N bench.py --gpus N ...        (one rank per GPU)

A step renders ONE full frame (3840x2160, 16 spheres, 3 lights, depth 5 =
RTSTACK_MAXSIZE 6, 3x3 supersampling = 74.6 M primary rays) of the seeded
synthetic scene from a scene already resident in HBM.  With
N > 1 the frame's rows are dealt row-cyclically (8-row blocks) to the ranks
and rank 0 gathers them with one RCCL gather over xGMI and restores row order
on the device, so the step ends with the whole frame in rank 0's HBM (strong
scaling: fixed frame).  Rank 0 prints one JSON line.

Also reported: the kernel roofline (VALU issue; work = the VALU operations the
kernel EXECUTES, counted per wave by the counting build of the same kernel,
rtg_amd/work.py; the reference's brute-force test count x 25 flops beside it
as `reference_work`), end-to-end frame times (scene preparation + upload,
render, read-back, PPM bytes), the reference CPU path timed on a bounded
pixel sample on this host (cpu_baseline), and parity of the produced
frame/PPM against the reference's golden hashes.
"""
from __future__ import annotations

import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch  # first: owns the HIP runtime librtg.so binds to (see rtg_amd)
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
import rtg_amd as R  # noqa: E402
from rtg_amd import dist as rdist  # noqa: E402
from rtg_amd import work as rwork  # noqa: E402

METRIC = "Mpixels/s (primary rays) + frame ms at WxH, depth D; PPM max-abs-diff vs CPU"
GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.json")
CONFIGS = {  # name: (W, H, spheres, lights, depth)  — BASELINE.json configs
    "c1": (640, 480, 4, 1, 1),
    "c2": (1920, 1080, 8, 2, 3),
    "c3": (3840, 2160, 16, 3, 5),
    "c4": (7680, 4320, 32, 4, 5),
    "c5": (3840, 2160, 1024, 4, 7),
}
# VALU issue peak: 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz = one wave64 VALU
# instruction per 2 cycles per SIMD (MI355X_MICROARCH.md: CDNA4 SIMDs are
# 32 wide; its 157.3 TFLOPS FP32 spec counts an FMA as two flops, and parity
# with the reference forbids contraction, so 78.6 T op/s is this kernel's
# ceiling).  BASELINE.md's 39.3 T assumed SIMD-16, which gfx950 is not.
VALU_PEAK_TOPS = rwork.VALU_PEAK_TOPS
HBM_PEAK_GBS = 8000.0
FLOPS_PER_TEST = 25  # raySphere pre-branch ops, SURVEY.md §8d


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def canon_md5(fb: np.ndarray) -> str:
    b = fb.view(np.uint32).copy()
    b[np.isnan(fb)] = 0xFFC00000
    return hashlib.md5(b.tobytes()).hexdigest()


def cpu_threads() -> int:
    """Host threads for the multi-threaded CPU baseline: the CPUs this process
    may run on, capped at 16 (the GPU box's CPU share per GPU)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def cpu_baseline(name, sph, lg, W, H, S, budget_s):
    """The reference CPU path (oracle/_ref, compiled from the reference's own
    raytracer.h) over a seeded uniform random sample of the frame's pixels,
    on one host thread (the reference's main.cpp:404 loop is single-threaded)
    and on all host threads; falls back to the C restatement
    (rows) if the reference build is absent.  Each leg gets half of
    `budget_s`: the sample grows until one run fills half of it (C5's pixels
    cost ~1000x C3's).  The multi-threaded figure is the baseline; the
    frame time is extrapolated from the sample."""
    ref = os.path.join(ROOT, "oracle", "_ref", f"librtgref_S{S}.so")
    port = os.path.join(ROOT, "oracle", "build", "librtg_oracle.so")
    kind = "reference" if os.path.exists(ref) else "port"
    L = ctypes.CDLL(ref if kind == "reference" else port)
    P = lambda a: ctypes.c_void_p(a.ctypes.data) if a.size else None  # noqa: E731
    rng = np.random.default_rng(7)
    perm = rng.permutation(W * H).astype(np.uint32)  # a prefix of it is a uniform sample

    def run(n, threads):
        if kind == "reference":
            gids = np.sort(perm[:n])
            out = np.zeros((n, 3), np.float32)
            t0 = time.perf_counter()
            L.ref_render_pixels(P(sph), len(sph), P(lg), len(lg), W, H, ctypes.c_float(-4.0),
                                ctypes.c_float(3.0), P(gids), n, P(out), threads)
            return time.perf_counter() - t0, gids, out
        rows = np.sort(rng.choice(H, size=max(1, n // W), replace=False)).astype(np.uint32)
        out = np.zeros((len(rows), W, 3), np.float32)
        t0 = time.perf_counter()
        L.oracle_render_rows(P(sph), len(sph), P(lg), len(lg), W, H, ctypes.c_float(-4.0),
                             ctypes.c_float(3.0), S, P(rows), len(rows), P(out), threads, None)
        gids = (rows[:, None].astype(np.int64) * W + np.arange(W)).reshape(-1)
        return time.perf_counter() - t0, gids, out.reshape(-1, 3)

    def leg(threads, budget):
        # grow the sample until one run fills at least half the budget (a
        # short run on many threads is dominated by start-up and tail)
        n = 64 * threads
        while True:
            t, gids, out = run(n, threads)
            if t >= 0.5 * budget or n >= W * H:
                break
            n = int(min(W * H, n * min(16.0, max(2.0, 0.8 * budget / max(t, 1e-6)))))
        px = len(gids)
        return {"value": round(px / t / 1e6, 5), "unit": "Mpixels/s", "cores": threads,
                "kind": kind,
                "sample": f"{name}: {px} pixels drawn uniformly from the {W}x{H} frame (seed 7)"
                          f", {t:.1f} s on {threads} thread{'s' if threads > 1 else ''}",
                "frame_s_extrapolated": round(t * W * H / px, 1)}, gids, out

    T = cpu_threads()
    one, g1, o1 = leg(1, budget_s / 2)
    if T > 1:
        multi, gm, om = leg(T, budget_s / 2)
        multi["single_thread"] = one
        return multi, np.concatenate([g1, gm]), np.concatenate([o1, om])
    return one, g1, o1


def cpu_only(args):
    """BASELINE configs[0] (C1: 640x480, 4 spheres, 1 light, depth 1): the
    reference CPU path itself, no GPU.  The reference build (oracle/_ref,
    raytracer.h compiled in place) renders the WHOLE frame with the
    reference's loop (main.cpp:404-453) on one host thread and on all host
    threads (<= 16); the frame and its PPM (savePPM, main.cpp:43-91) are
    checked against the golden md5s.  One JSON line, n_gpus 0."""
    W, H, n, m, depth = CONFIGS[args.config]
    S = depth + 1
    ref = os.path.join(ROOT, "oracle", "_ref", f"librtgref_S{S}.so")
    if not os.path.exists(ref):
        raise SystemExit(f"cpu-only: the reference build {ref} is missing (oracle/build_ref.sh)")
    L = ctypes.CDLL(ref)
    sph, lg = R.generate_scene(n, m, 42)
    P = lambda a: ctypes.c_void_p(a.ctypes.data) if a.size else None  # noqa: E731
    rows = np.arange(H, dtype=np.uint32)
    golden = json.load(open(GOLDEN))["configs"].get(args.config, {})
    legs = {}
    for threads in sorted({1, cpu_threads()}):
        times = []
        for _ in range(max(1, args.steps)):
            fb = np.zeros((H, W, 3), np.float32)
            t0 = time.perf_counter()
            L.ref_render_rows(P(sph), n, P(lg), m, W, H, ctypes.c_float(-4.0),
                              ctypes.c_float(3.0), P(rows), H, P(fb), threads)
            times.append(time.perf_counter() - t0)
        med = float(np.median(times))
        mx = R.max_colour_value(fb)
        ppm = R.ppm_file_bytes(fb, mx)
        legs[threads] = {"frame_ms": round(med * 1e3, 3), "value": round(W * H / med / 1e6, 3),
                         "cores": threads, "runs": len(times),
                         "fb_md5_match": canon_md5(fb) == golden.get("fb_md5"),
                         "ppm_md5_match": hashlib.md5(ppm).hexdigest() == golden.get("ppm_md5")}
    if args.ppm_out:
        with open(args.ppm_out, "wb") as f:
            f.write(ppm)
    best = legs[max(legs)]
    out = {"metric": METRIC, "value": best["value"], "unit": "Mpixels/s", "n_gpus": 0,
           "steps": max(1, args.steps), "warmup": 0, "ms_per_step": best["frame_ms"],
           "higher_is_better": True, "scaling": "none", "vs_baseline": None, "dtype": "f32",
           "data": "synthetic: seeded scene generator (SURVEY.md §8d, seed 42)",
           "config": {"workload": f"{args.config}: {W}x{H}, {n} spheres, {m} lights, depth "
                                  f"{depth}: the reference CPU path (raytracer.h), PPM out, no GPU",
                      "width": W, "height": H, "spheres": n, "lights": m, "depth": depth},
           "cpu_only": True,
           "cpu_baseline": {"kind": "reference", "unit": "Mpixels/s", **best,
                            "sample": f"{args.config}: the whole {W}x{H} frame, median of "
                                      f"{best['runs']} runs",
                            "single_thread": legs[1]},
           "parity": {"fb_md5_match": best["fb_md5_match"] and legs[1]["fb_md5_match"],
                      "ppm_md5_match": best["ppm_md5_match"] and legs[1]["ppm_md5_match"],
                      "reference": "tests/golden (reference raytracer.h output)"}}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--row-block", type=int, default=8,
                    help="rows per block of the row-cyclic deal (8: <1 %% imbalance at 8 ranks on C3)")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--ab", default="", help="comma list of kernel variants to A/B after the "
                    "timed run (interleaved rounds, kernel time via HIP events)")
    ap.add_argument("--ab-rounds", type=int, default=5)
    ap.add_argument("--diag", type=int, default=0, help="diagnostic variant (e.g. 102) to run "
                    "once after timing; reports s_memtime cycle shares per phase")
    ap.add_argument("--cpu-budget", type=float, default=16.0,
                    help="seconds of CPU baseline (split between the 1-thread and all-thread legs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-work-count", action="store_true",
                    help="skip the counting-build run (executed-work roofline); PMC passes use "
                         "this so that only the timed kernel is profiled")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end frame timings")
    ap.add_argument("--gather-chunks", type=int, default=0,
                    help="N > 1: split each rank's rows into K chunks; each chunk is rendered "
                         "then gathered asynchronously, so RCCL overlaps the next chunk's "
                         "rendering (1 = render all, then one gather; 0 = by world size, "
                         "rtg_amd.dist.default_chunks)")
    ap.add_argument("--last-chunk-frac", type=float, default=-1.0,
                    help="N > 1: the last chunk's share of the shard (0 = equal chunks; "
                         "negative = by world size)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: gather through host memory (lets N ranks share one GPU "
                         "to exercise the multi-rank path on a 1-GPU box)")
    ap.add_argument("--cpu-only", action="store_true",
                    help="BASELINE configs[0]: time the reference CPU path on the whole frame "
                         "(no GPU), check its frame and PPM md5s; with --config c1")
    ap.add_argument("--ppm-out", default="", help="--cpu-only: write the PPM here")
    args = ap.parse_args()
    if args.cpu_only:
        cpu_only(args)
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    ndev = torch.cuda.device_count()
    local = local % max(ndev, 1)  # only differs when ranks share a GPU (gloo rehearsal)
    torch.cuda.set_device(local)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    W, H, n, m, depth = CONFIGS[args.config]
    S = depth + 1
    B = args.row_block
    sph, lg = R.generate_scene(n, m, 42)
    ctx = R.Context(local)
    t_scene = []
    for _ in range(3 if world == 1 else 1):  # host preparation + upload, blocking
        t0 = time.perf_counter()
        ctx.set_scene(sph, lg)
        t_scene.append((time.perf_counter() - t0) * 1e3)
    scene_stats = ctx.scene_stats()
    if args.variant:
        ctx.set_variant(args.variant)

    Rmax = rdist.padded_rows(H, B, world)
    my_rows = R.shard_rows(H, B, rank, world)
    shard = torch.zeros((Rmax, W, 3), dtype=torch.float32, device="cuda")
    frame_buf = (torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
                 if (world > 1 and rank == 0) else None)
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream
    ev_k = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            for _ in range(args.steps)]
    # N > 1, rank 0: gather complete (after the waits) and assemble done
    # N > 1, rank 0, all on the assembling stream (so their order is the
    # stream's): every chunk rendered, the last chunk gathered, assembled
    ev_r = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev_g = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev_a = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    # N > 1: chunks of the padded shard, whole row blocks (same row ranges on
    # every rank); chunk c's rows of all ranks are global rows [r0 G, r1 G),
    # gathered into their own [world, r1 - r0] buffer and put in row order by
    # the assemble kernel as soon as that chunk has arrived.  The global rows
    # of this rank's real rows, for rtg_render_rows_device.
    nblk = Rmax // B
    auto_k, auto_f = rdist.default_chunks(world)
    K = max(1, min(args.gather_chunks or auto_k, nblk)) if world > 1 else 1
    last_frac = args.last_chunk_frac if args.last_chunk_frac >= 0.0 else auto_f
    bounds = rdist.chunk_bounds(nblk, K, B, last_frac if world > 1 else 0.0)
    gathered = ([torch.empty((world, bounds[c + 1] - bounds[c], W, 3), dtype=torch.float32,
                             device="cuda") for c in range(K)]
                if (world > 1 and rank == 0) else None)
    grow = torch.tensor(R.shard_row_indices(H, B, rank, world).astype(np.int64),
                        dtype=torch.int32, device="cuda") if world > 1 else None
    # chunks render on two streams in turn, so one chunk's last waves overlap
    # the next chunk's first ones (a launch ends with a tail of long waves);
    # rank 0 restores each chunk's row order on a third stream as soon as that
    # chunk has arrived, overlapping the later chunks' rendering
    rstreams = [torch.cuda.Stream(), torch.cuda.Stream()] if world > 1 else None
    astream = torch.cuda.Stream() if (world > 1 and rank == 0) else None

    frame = None

    # N = 1: the launches run back to back and two HIP events bracket the whole
    # timed region (per-launch events add a timestamp packet between kernels);
    # N > 1: events bracket each step's render chunks.
    ev_region = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))

    def step(i=None):
        nonlocal frame
        if world == 1:
            ctx.render_device(W, H, shard.data_ptr(), stack_size=S, row_block=B, shard=0,
                              n_shards=1, stream=sptr)
            frame = shard[:H]
            return
        if i is not None:
            ev_k[i][0].record(stream)
        for rs in rstreams:
            rs.wait_stream(stream)
        if astream is not None:
            astream.wait_stream(stream)
        works = []
        for c in range(K):
            r0, r1 = bounds[c], bounds[c + 1]
            nreal = max(0, min(r1, my_rows) - r0)
            rs = rstreams[c % 2]
            with torch.cuda.stream(rs):
                if nreal > 0:
                    ctx.render_rows_device(W, H, grow.data_ptr() + 4 * r0, nreal,
                                           shard.data_ptr() + 12 * W * r0, stack_size=S,
                                           stream=rs.cuda_stream)
                piece = shard[r0:r1]
                if args.dist_backend == "nccl":  # RCCL gather over xGMI, overlapped
                    outs = [gathered[c][g] for g in range(world)] if rank == 0 else None
                    works.append(dist.gather(piece, outs, dst=0, async_op=True))
                else:                            # rehearsal path through host memory
                    host = piece.cpu()
                    gl = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
                    dist.gather(host, gl, dst=0)
                    if rank == 0:
                        for g in range(world):
                            gathered[c][g].copy_(gl[g])
                    works.append(None)
            if astream is not None:  # rank 0: chunk c in row order once it has arrived
                with torch.cuda.stream(astream):
                    if i is not None and c == K - 1:  # every chunk rendered (both streams)
                        for rs_ in rstreams:
                            astream.wait_stream(rs_)
                        ev_r[i].record(astream)
                    if works[c] is not None:
                        works[c].wait()  # astream waits for chunk c's gather
                    else:
                        astream.wait_stream(rs)  # the host-memory copies above
                    if i is not None and c == K - 1:
                        ev_g[i].record(astream)
                    hc = min(H - r0 * world, (r1 - r0) * world)
                    if hc > 0:  # native permute kernel, at global row r0 G
                        ctx.assemble_shards_device(gathered[c].data_ptr(), world, r1 - r0, W, hc,
                                                   B, frame_buf.data_ptr() + 12 * W * r0 * world,
                                                   stream=astream.cuda_stream)
        for rs in rstreams:
            stream.wait_stream(rs)
        if i is not None:
            ev_k[i][1].record(stream)
        if astream is not None:
            if i is not None:
                ev_a[i].record(astream)
            stream.wait_stream(astream)
        else:
            for w in works:  # the shard is rendered into again next step
                if w is not None:
                    w.wait()
        if rank == 0:
            frame = frame_buf

    # The first launch after set_scene (no launch-order feedback yet: the
    # reference's single enqueue + clFinish, main.cpp:353-374), timed alone:
    # the process's very first launch (code objects loaded, launch scratch
    # allocated: first_launch_process_ms), then set_scene again (a new scene
    # generation, so no feedback) and its first launch (first_launch_ms).
    first_ms = first_proc_ms = None
    if world == 1:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for k in range(2):
            if k == 1:
                ctx.set_scene(sph, lg)
            torch.cuda.synchronize()
            e0.record(stream)
            step()
            e1.record(stream)
            torch.cuda.synchronize()
            if k == 0:
                first_proc_ms = e0.elapsed_time(e1)
            else:
                first_ms = e0.elapsed_time(e1)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_region[0].record(stream)
    for i in range(args.steps):
        step(i)
    ev_region[1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world == 1:  # mean kernel time over the timed region (launches back to back)
        kern_ms = ev_region[0].elapsed_time(ev_region[1]) / args.steps
    else:
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev_k]))
    multi = None
    if world > 1:
        dev = "cuda" if args.dist_backend == "nccl" else "cpu"
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_max_ms = float(t[0]), float(t[1])
        # every rank's render time (its shard's chunks, HIP events), on rank 0
        mine = torch.tensor([kern_ms], dtype=torch.float64, device=dev)
        allr = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [round(float(x[0]), 4) for x in allr]
        if rank == 0:  # its events, all on the assembling stream (non-negative)
            gather_tail = float(np.mean([ev_r[i].elapsed_time(ev_g[i])
                                         for i in range(args.steps)]))
            assemble = float(np.mean([ev_g[i].elapsed_time(ev_a[i]) for i in range(args.steps)]))
        else:
            gather_tail = assemble = 0.0
        multi = {"render_ms_per_rank": per_rank,
                 "render_imbalance": round(max(per_rank) / (sum(per_rank) / world), 4),
                 "gather_tail_ms_rank0": round(gather_tail, 4),
                 "assemble_ms_rank0": round(assemble, 4),
                 "step_ms": round(elapsed / args.steps * 1e3, 4),
                 "gather_chunks": K,
                 "chunk_rows": [bounds[c + 1] - bounds[c] for c in range(K)],
                 "note": "render = this rank's shard chunks (HIP events, chunks on two "
                         "streams in turn); gather tail = rank 0's last chunk rendered to the "
                         "last chunk gathered, both events on its assembling stream (earlier "
                         "chunks' gathers and assembles "
                         "overlap rendering); assemble = the last chunk's arrival to the end of "
                         "its row-order restore on rank 0 (each chunk is restored on a third "
                         "stream as it arrives); step = wall time per frame, max over ranks"}
    else:
        kern_max_ms = kern_ms

    ms_per_step = elapsed / args.steps * 1e3
    mpx = W * H / (elapsed / args.steps) / 1e6

    # The first launches of a fresh frame geometry on a WARM GPU (after the
    # timed region; set_scene starts a new scene generation, so the launch-
    # order feedback starts empty).  first_launch_ms above is the same launch
    # at process start, where the GPU is still ramping its clocks: the cold
    # probe (tools/cold_probe.py, profiles/r05/cold_probe_c3.txt) puts the
    # feedback-ordered steady launch at process start ~20 % above the warm one,
    # so the two figures separate the launch path's own cold cost from the
    # GPU's power-state ramp.
    fresh_ms = None
    if world == 1:
        fresh_ms = []
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ctx.set_scene(sph, lg)
        for _ in range(3):
            torch.cuda.synchronize()
            e0.record(stream)
            step()
            e1.record(stream)
            torch.cuda.synchronize()
            fresh_ms.append(round(e0.elapsed_time(e1), 4))

    diag = None
    if args.diag and world == 1:
        ctx.set_variant(args.diag)
        ctx.diag_read(reset=True)
        ctx.render_device(W, H, shard.data_ptr(), stack_size=S, row_block=B, stream=sptr)
        torch.cuda.synchronize()
        cyc = ctx.diag_read(reset=True)
        tot = max(cyc[3], 1)
        names = ["closest", "shadow", "refraction", "total", "matte", "push", "unwind", "shade"]
        diag = {"variant": args.diag, "wave_cycles_total": cyc[3]}
        for k, nm in enumerate(names):
            if k != 3:
                diag["share_" + nm] = round(cyc[k] / tot, 4)
        diag["share_outside_closest_shade_unwind"] = round(
            1 - (cyc[0] + cyc[7] + cyc[6]) / tot, 4)
        log("diag", diag)
        ctx.set_variant(args.variant)

    ab = None
    if args.ab and world == 1:
        variants = [int(v) for v in args.ab.split(",")]
        times = {v: [] for v in variants}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(args.ab_rounds):
            for v in variants:
                ctx.set_variant(v)
                ctx.render_device(W, H, shard.data_ptr(), stack_size=S, row_block=B,
                                  stream=sptr)  # warm
                e0.record(stream)
                for _ in range(3):
                    ctx.render_device(W, H, shard.data_ptr(), stack_size=S, row_block=B,
                                      stream=sptr)
                e1.record(stream)
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1) / 3)
        ctx.set_variant(args.variant)
        ab = {str(v): {"median_ms": round(float(np.median(t)), 4),
                       "min_ms": round(float(np.min(t)), 4)} for v, t in times.items()}
        log("A/B", ab)

    if rank != 0:
        dist.destroy_process_group()
        return

    # ---------------- parity of the produced frame vs the reference goldens
    golden = json.load(open(GOLDEN)) if os.path.exists(GOLDEN) else {"configs": {}}
    g = golden["configs"].get(args.config, {})
    fb = frame.cpu().numpy()
    parity = {"reference": "tests/golden (reference raytracer.h output)"}
    if "fb_md5" in g:
        got = canon_md5(fb)
        parity["fb_md5_match"] = got == g["fb_md5"]
        mx = R.max_colour_value(fb)
        ppm = R.ppm_file_bytes(fb, mx)
        parity["ppm_md5_match"] = hashlib.md5(ppm).hexdigest() == g["ppm_md5"]
        parity["max_colour_match"] = int(np.float32(mx).view(np.uint32)) == g["max_colour_bits"]
    # max-abs-diff vs the reference CPU path on golden rows (and CPU sample below)
    rows_file = os.path.join(ROOT, "tests", "golden", f"{args.config}.rows.f32")
    diffs = []
    if "rows" in g and os.path.exists(rows_file):
        rows = g["rows"]["rows"]
        want = np.fromfile(rows_file, np.float32).reshape(len(rows), W, 3)
        diffs.append((fb[rows], want))
    if "wide" in g:  # C5's widened reference sample (tests/golden/make_c5_wide.py)
        z = np.load(os.path.join(ROOT, "tests", "golden", g["wide"]["file"]))
        diffs.append((fb[z["rows"].astype(np.int64)], z["rows_fb"]))
        diffs.append((fb.reshape(-1, 3)[z["gids"].astype(np.int64)], z["pixels"]))

    # ---------------- CPU baseline (rank 0, N = 1 only)
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu, cgid, cout = cpu_baseline(args.config, sph, lg, W, H, S, args.cpu_budget)
        diffs.append((fb.reshape(-1, 3)[cgid], cout))
    if diffs:
        a = np.concatenate([d[0].reshape(-1) for d in diffs])
        b = np.concatenate([d[1].reshape(-1) for d in diffs])
        nan_a, nan_b = np.isnan(a), np.isnan(b)
        ok = ~(nan_a | nan_b)
        parity["max_abs_diff_float"] = float(np.max(np.abs(a[ok] - b[ok]))) if ok.any() else 0.0
        parity["nan_positions_match"] = bool((nan_a == nan_b).all())
        parity["bit_exact"] = bool(parity["nan_positions_match"] and np.array_equal(
            a[ok].view(np.uint32), b[ok].view(np.uint32)))
        parity["values_compared"] = int(a.size)
        # PPM bytes of those pixels under the frame's max colour
        mx = R.max_colour_value(fb)
        pa, pb = R.ppm_bytes(a.reshape(-1, 3), mx), R.ppm_bytes(b.reshape(-1, 3), mx)
        parity["ppm_max_abs_diff"] = int(np.max(np.abs(pa.astype(int) - pb.astype(int))))

    # ---------------- executed work (counting build of the timed kernel)
    # Variant 120 runs the default kernel's control flow with per-wave unit
    # counters (rtg_amd/work.py); one frame, after the timed region.
    work = None
    if world == 1 and not args.no_work_count and args.variant == 0:
        ctx.set_variant(120)
        ctx.diag_counts(reset=True)
        ctx.render_device(W, H, shard.data_ptr(), stack_size=S, row_block=B, stream=sptr)
        torch.cuda.synchronize()
        wv, lv = ctx.diag_counts(reset=True)
        ctx.set_variant(args.variant)
        work = rwork.executed_work(R.UNIT_NAMES, wv, lv)
        work["counters"] = {nm: [int(wv[k]), int(lv[k])] for k, nm in enumerate(R.UNIT_NAMES)
                            if not nm.startswith("U.")}

    # ---------------- end to end (N = 1): the reference's per-run flow
    e2e = None
    if world == 1 and not args.no_e2e:
        host = torch.empty((H, W, 3), dtype=torch.float32, pin_memory=True)
        mxd = torch.empty(1, dtype=torch.float32, device="cuda")
        ppm_d = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
        ppm_h = torch.empty(H * W * 3, dtype=torch.uint8, pin_memory=True)
        t_full, t_d2h, t_ppm, t_cold = [], [], [], []
        c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            # scene upload (main.cpp:277-294) + render and finish (:353-374) +
            # read-back of the float frame (:460); the render is the first
            # after set_scene (no launch-order feedback)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.set_scene(sph, lg)
            c0.record(stream)
            ctx.render_device(W, H, shard.data_ptr(), stack_size=S, row_block=B, stream=sptr)
            c1.record(stream)
            torch.cuda.synchronize()
            t_cold.append(c0.elapsed_time(c1))
            t1 = time.perf_counter()
            host.copy_(shard[:H], non_blocking=True)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            t_full.append((t2 - t0) * 1e3)
            t_d2h.append((t2 - t1) * 1e3)
            # resident scene: render, device max + PPM bytes (algebra.h:68-91,
            # main.cpp:66-81), read-back of the 3 B/px image
            t0 = time.perf_counter()
            ctx.render_device(W, H, shard.data_ptr(), stack_size=S, row_block=B, stream=sptr)
            ctx.max_colour_device(shard.data_ptr(), W * H, mxd.data_ptr(), stream=sptr)
            ctx.ppm_bytes_device(shard.data_ptr(), W * H, mxd.data_ptr(), ppm_d.data_ptr(),
                                 stream=sptr)
            ppm_h.copy_(ppm_d, non_blocking=True)
            torch.cuda.synchronize()
            t_ppm.append((time.perf_counter() - t0) * 1e3)
        e2e = {"e2e_ms": round(float(np.median(t_full)), 3),
               "scene_prep_ms": round(float(np.median(t_scene)), 3),
               "scene_host_prep_ms": round(scene_stats["prep_ms"], 3),
               "scene_upload_ms": round(scene_stats["upload_ms"], 3),
               "scene_device_bytes": scene_stats["device_bytes"],
               "bvh_nodes": scene_stats["bvh_nodes"],
               "render_ms": round(float(np.median(t_cold)), 4),
               "render_fed_ms": round(kern_ms, 4),
               "d2h_fb_ms": round(float(np.median(t_d2h)), 3),
               "e2e_ppm_resident_scene_ms": round(float(np.median(t_ppm)), 3),
               "note": "e2e_ms = set_scene (host masks/BVH + H2D) + render (the first after "
                       "set_scene, no launch-order feedback: render_ms) + D2H of the "
                       f"{W * H * 12 / 1e6:.1f} MB float frame into pinned memory (main.cpp:277-"
                       "294, 353-374, 460); e2e_ppm_resident_scene_ms = render + device max + "
                       "PPM bytes + D2H of 3 B/px; medians of 3"}

    # ---------------- roofline (rank-0 launch)
    tests = g.get("ray_sphere_tests")
    roof = None
    hbm = {"achieved_GBs": round(my_rows * W * 12 / (kern_ms * 1e-3) / 1e9, 2),
           "peak_GBs": HBM_PEAK_GBS,
           "frac": round(my_rows * W * 12 / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6),
           "algorithmic_bytes": my_rows * W * 12}
    if work is not None:
        ach = work["lane_ops"] / (kern_ms * 1e-3) / 1e12
        roof = {"bound": "valu", "achieved": round(ach, 3), "peak": round(VALU_PEAK_TOPS, 1),
                "unit": "TFLOP/s", "frac": round(ach / VALU_PEAK_TOPS, 4), "traffic": None,
                "work": f"{work['lane_ops']:.4g} executed VALU lane-ops per frame = 64 x "
                        f"{work['valu_slots']:.4g} wave-instruction slots, counted per wave by "
                        "the counting build (variant 120) and priced per unit "
                        "(rtg_amd/work.py), / mean kernel time "
                        f"{kern_ms:.3f} ms (HIP events on the launch stream)",
                "executed_valu_slots": work["valu_slots"],
                "units": {k: v for k, v in sorted(work["units"].items(),
                                                  key=lambda kv: -kv[1]["slots"]) if v["waves"]},
                "counters": work["counters"],
                "hbm": hbm}
        if tests:
            roof["reference_work"] = {
                "flop": tests * FLOPS_PER_TEST,
                "note": f"{tests} ray-sphere tests of the reference's brute-force scans x "
                        f"{FLOPS_PER_TEST} FP32 ops (SURVEY.md §8d)"}
            roof["work_avoided_ratio"] = round(tests * FLOPS_PER_TEST / work["lane_ops"], 3)
    elif tests:  # no counting run: the reference's test count only, labelled as such
        flops = tests * FLOPS_PER_TEST * my_rows / H
        roof = {"bound": "valu", "achieved": None, "peak": round(VALU_PEAK_TOPS, 1),
                "unit": "TFLOP/s", "frac": None, "traffic": None,
                "reference_work": {"flop": flops, "per_s_T": round(flops / (kern_ms * 1e-3) / 1e12, 3),
                                   "note": "reference brute-force tests x 25 (not executed work)"},
                "hbm": hbm}
    if roof is not None:
        # HBM traffic and VALU issue per launch from the committed PMC passes
        # (tools/gpu_pmc.sh -> profiles/pmc_<config>.json), used only when
        # measured on these kernel sources, this variant and N = 1.
        pmc = os.path.join(ROOT, "profiles", f"pmc_{args.config}.json")
        if os.path.exists(pmc) and world == 1:
            rec = json.load(open(pmc))
            import importlib.util
            spec = importlib.util.spec_from_file_location(
                "pmc_summary", os.path.join(ROOT, "tools", "pmc_summary.py"))
            mod = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(mod)
            if rec.get("source_md5") == mod.source_md5() and rec.get("variant") == args.variant \
                    and "traffic_bytes" in rec:
                roof["traffic"] = int(rec["traffic_bytes"])
                if "valu_issue_utilisation" in rec:
                    roof["valu_issue_utilisation_pmc"] = round(rec["valu_issue_utilisation"], 3)
                vi = rec.get("counters", {}).get("SQ_INSTS_VALU")
                if vi and work is not None:
                    roof["pmc_valu_insts"] = int(vi)
                    roof["model_vs_pmc_valu"] = round(work["valu_slots"] / vi, 3)
                    # the unit prices are FITTED to SQ_INSTS_VALU over a scene
                    # set that includes the bench configs (tools/calib_units.py),
                    # so this ratio is in-sample; the held-out figures are in
                    # the fit record
                    roof["model_vs_pmc_valu_kind"] = (
                        "fitted (in sample); held-out ratios: rtg_amd/work.py FIT_RECORD")
                if vi:
                    # the same roofline from the hardware's count of executed
                    # VALU wave instructions (x 64 lanes) per launch, over this
                    # run's mean kernel time.  It is the headline `frac` when
                    # present (instruction counts are the same on any box for
                    # these sources and this frame); the counting model's
                    # stays beside it (frac_model) with its per-unit split.
                    ach_pmc = vi * 64 / (kern_ms * 1e-3) / 1e12
                    roof["achieved_pmc"] = round(ach_pmc, 3)
                    roof["frac_pmc"] = round(ach_pmc / VALU_PEAK_TOPS, 4)
                    if roof.get("frac") is not None:
                        roof["achieved_model"] = roof["achieved"]
                        roof["frac_model"] = roof["frac"]
                    roof["achieved"] = roof["achieved_pmc"]
                    roof["frac"] = roof["frac_pmc"]
                    roof["frac_source"] = ("PMC SQ_INSTS_VALU x 64 per launch "
                                           f"({os.path.relpath(pmc, ROOT)}) / mean kernel time "
                                           f"{kern_ms:.4f} ms (HIP events)")
                roof["traffic_note"] = ("PMC FETCH_SIZE x2 + WRITE_SIZE per launch "
                                        f"({os.path.relpath(pmc, ROOT)})")

    out = {
        "metric": METRIC, "value": round(mpx, 2), "unit": "Mpixels/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: seeded scene generator (SURVEY.md §8d, seed 42), resident in HBM",
        "config": {"workload": f"{args.config}: {W}x{H}, {n} spheres, {m} lights, depth {depth} "
                               f"(RTSTACK_MAXSIZE {S}), 3x3 supersampling",
                   "width": W, "height": H, "spheres": n, "lights": m, "depth": depth,
                   "alias_factor": 3, "row_block": B, "variant": args.variant,
                   "parallelism": f"row-cyclic x{world}" + (
                       ((f" + RCCL gather ({K} pipelined chunks)") if args.dist_backend == "nccl"
                        else " + gloo gather") if world > 1 else "")},
        "mrays_per_s": round(mpx * 9, 1),
        "kernel_ms": round(kern_ms, 4), "kernel_ms_max_rank": round(kern_max_ms, 4),
        "first_launch_ms": round(first_ms, 4) if first_ms is not None else None,
        "first_launch_process_ms": round(first_proc_ms, 4) if first_proc_ms is not None else None,
        "first_launch_warm_gpu_ms": fresh_ms[0] if fresh_ms else None,
        "fresh_geometry_launches_warm_ms": fresh_ms,
        "timed_launches": {"first": 2 + args.warmup if world == 1 else None,
                           "count": args.steps,
                           "note": "trace-kernel dispatches [first, first + count) of this "
                                   "process are the timed region's (tools/timed_stats.py)"},
        "roofline": roof, "cpu_baseline": cpu, "e2e": e2e, "multi_gpu": multi,
        "gpu_vs_cpu": round(mpx / cpu["value"], 1) if cpu else None,
        "parity": parity,
        "ab": ab,
        "diag": diag,
    }
    print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
