"""GPU parity tests: the HIP kernel (through the C ABI) against the
reference-generated golden fixtures and the oracle, on an MI355X.

Bar: every non-NaN float bit-identical, NaNs at the same positions (the
kernel writes the x86 default NaN 0xFFC00000); PPM bytes identical.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import pytest

from conftest import (GOLDEN, bits_equal, canon_md5, first_mismatch, load_f32, load_scene, md5,
                      random_scene)

pytestmark = pytest.mark.gpu

ALL = ["ref800", "c1", "c2", "c3", "c4", "c5"]
# Kernel variants of the shipped librtg.so (rtg_trace_kernels.h kVariants);
# the A/B variants exist only in `make AB=1` builds (test_ab_variants).
SHIPPED = [0, 9, 100, 110, 120]
AB_VARIANTS = [1, 2, 3, 4, 5, 6, 8, 14, 15, 18, 19, 20, 21, 22, 23, 24, 104, 108]


@pytest.fixture(scope="module")
def R(rtg):
    if rtg.device_count() < 1:
        pytest.fail("no GPU visible to librtg")
    return rtg


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    assert torch.cuda.is_available()
    return torch


def test_device_info(R):
    info = R.device_info(0)
    assert "gfx950" in info, info


@pytest.mark.parametrize("name", ALL)
def test_small_frames(R, golden, name):
    c = golden["configs"][name]
    sph, lg = load_scene(name, c["spheres"], c["lights"])
    sw, sh = c["small"]["W"], c["small"]["H"]
    want = load_f32(os.path.join(GOLDEN, f"{name}.small.f32"), (sh, sw, 3))
    got = R.render(sph, lg, sw, sh, stack_size=c["stack_size"])
    assert bits_equal(got, want), first_mismatch(got, want)
    # NaNs come out as the x86 default NaN
    nan = np.isnan(got)
    assert (got.view(np.uint32)[nan] == 0xFFC00000).all()


def test_edge_cases(R, golden):
    for c in golden["cases"]:
        sph, lg = load_scene(c["name"], c["spheres"], c["lights"])
        want = load_f32(os.path.join(GOLDEN, c["name"] + ".f32"), (c["H"], c["W"], 3))
        got = R.render(sph, lg, c["W"], c["H"], zoom=c["zoom"], alias_factor=c["aliasFactor"],
                       stack_size=c["stack_size"])
        assert bits_equal(got, want), (c["name"], first_mismatch(got, want))


@pytest.mark.parametrize("name", ["ref800", "c1", "c2", "c3", "c4", "c5"])
def test_full_frames_md5_and_ppm(R, golden, tmp_path, name):
    """Whole frames against the reference's: canonical-bits md5, NaN count,
    sampled rows, max colour and PPM md5 (C5's whole frame from
    tests/golden/make_c5_full.py: the reference build over all 2160 rows)."""
    c = golden["configs"][name]
    if "fb_md5" not in c:
        pytest.skip("golden has no full frame for " + name)
    sph, lg = load_scene(name, c["spheres"], c["lights"])
    fb = R.render(sph, lg, c["W"], c["H"], stack_size=c["stack_size"])
    assert canon_md5(fb) == c["fb_md5"], name
    assert int(np.isnan(fb).sum()) == c["nan_values"]
    rows = c["rows"]["rows"]
    want = load_f32(os.path.join(GOLDEN, f"{name}.rows.f32"), (len(rows), c["W"], 3))
    assert bits_equal(fb[rows], want)
    mx = R.max_colour_value(fb)
    assert np.float32(mx).view(np.uint32) == c["max_colour_bits"]
    path = str(tmp_path / f"{name}.ppm")
    R.save_ppm(fb, path, mx)
    assert md5(open(path, "rb").read()) == c["ppm_md5"]


def test_c5_sampled_rows(R, golden):
    """1024 spheres, depth 7: the LDS-spill stress config (sampled rows)."""
    c = golden["configs"]["c5"]
    sph, lg = load_scene("c5", c["spheres"], c["lights"])
    rows = c["rows"]["rows"]
    want = load_f32(os.path.join(GOLDEN, "c5.rows.f32"), (len(rows), c["W"], 3))
    got = R.render_rows(sph, lg, c["W"], c["H"], rows, stack_size=c["stack_size"])
    assert bits_equal(got, want), first_mismatch(got, want)


def test_c5_wide_sample(R, golden, torch_cuda):
    """C5 against the widened reference fixture (tests/golden/make_c5_wide.py):
    85 full-width rows (every 32nd, the centre band 1072..1087, the last) and
    100,000 seeded random pixels of the whole frame, from one full-frame
    render of the default (BVH) kernel."""
    torch = torch_cuda
    c = golden["configs"]["c5"]
    wide = c["wide"]
    z = np.load(os.path.join(GOLDEN, wide["file"]))  # allow_pickle=False (default)
    rows, want_rows, gids, want_px = z["rows"], z["rows_fb"], z["gids"], z["pixels"]
    assert len(rows) == wide["rows"] and len(gids) == wide["pixels"]
    assert canon_md5(want_rows) == wide["rows_md5"] and canon_md5(want_px) == wide["pixels_md5"]
    sph, lg = load_scene("c5", c["spheres"], c["lights"])
    W, H = c["W"], c["H"]
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    ctx.render_device(W, H, out.data_ptr(), stack_size=c["stack_size"],
                      stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    fb = out.cpu().numpy()
    ctx.close()
    got_rows = fb[rows.astype(np.int64)]
    assert bits_equal(got_rows, want_rows), first_mismatch(got_rows, want_rows)
    got_px = fb.reshape(-1, 3)[gids.astype(np.int64)]
    assert bits_equal(got_px, want_px), first_mismatch(got_px, want_px)
    # the old 5-row fixture agrees with the same frame
    old = load_f32(os.path.join(GOLDEN, "c5.rows.f32"), (len(c["rows"]["rows"]), W, 3))
    assert bits_equal(fb[c["rows"]["rows"]], old)


def test_random_scenes_vs_oracle(R, oracle):
    rng = np.random.default_rng(2026)
    for trial in range(24):
        S = int(rng.integers(1, 17))
        n, m = int(rng.integers(0, 20)), int(rng.integers(0, 5))
        W, H = int(rng.integers(1, 70)), int(rng.integers(1, 50))
        aa = float(rng.choice([1.0, 2.0, 3.0, 2.5, 4.0]))
        zoom = float(rng.choice([-4.0, -2.0, -7.0, 3.0, 0.5]))
        sph, lg = random_scene(rng, n, m)
        if zoom > 0:
            sph["pos"][:, 2] *= -1.0
        want = oracle.render(sph, lg, W, H, S, aa=aa, zoom=zoom)
        got = R.render(sph, lg, W, H, zoom=zoom, alias_factor=aa, stack_size=S)
        assert bits_equal(got, want), (trial, S, n, m, W, H, first_mismatch(got, want))


def _random_vs_oracle(R, oracle, torch, variant, trials=16):
    rng = np.random.default_rng(77 + variant)
    ctx = R.Context(0)
    ctx.set_variant(variant)
    for trial in range(trials):
        S = int(rng.integers(1, 17))
        n, m = int(rng.integers(0, 20)), int(rng.integers(0, 5))
        W, H = int(rng.integers(1, 70)), int(rng.integers(1, 50))
        aa = float(rng.choice([0.5, 1.0, 2.0, 3.0, 2.5, 4.0, 5.0, 8.0, 9.0]))
        zoom = float(rng.choice([-4.0, -2.0, 3.0]))
        sph, lg = random_scene(rng, n, m)
        if zoom > 0:
            sph["pos"][:, 2] *= -1.0
        want = oracle.render(sph, lg, W, H, S, aa=aa, zoom=zoom)
        ctx.set_scene(sph, lg)
        out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        ctx.render_device(W, H, out.data_ptr(), zoom=zoom, alias_factor=aa, stack_size=S,
                          stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert bits_equal(got, want), (trial, S, n, m, W, H, aa, first_mismatch(got, want))
    ctx.close()


@pytest.mark.parametrize("variant", [0, 9])
def test_random_scenes_vs_oracle_variants(R, oracle, torch_cuda, variant):
    """The sample kernel and the tile kernel over random scenes, sizes and
    alias factors (the sample-parallel kernel packs 64 // nAA^2 pixels per
    wave and falls back to the tile kernel above nAA = 8)."""
    _random_vs_oracle(R, oracle, torch_cuda, variant)


def clustered_scene(rng, n, m, refr_frac=0.5):
    """A BVH-scale scene (n > 64): spheres packed in a few overlapping
    clusters, many of them refractive, several lights, so that the coherent
    waves take the sphere lists (capsule / overlap lists) and the incoherent
    ones the BVH queries."""
    import rtg_amd as R
    sph = np.zeros(n, R.SPHERE_DTYPE)
    k = int(rng.integers(2, 5))
    ctr = np.stack([rng.uniform(-8, 8, k), rng.uniform(-5, 5, k), rng.uniform(-30, -10, k)], 1)
    for i in range(n):
        c = ctr[int(rng.integers(0, k))]
        sph[i]["pos"] = c + rng.normal(0, 3.0, 3)
        sph[i]["radius"] = rng.uniform(0.2, 1.6)
        op = 0.0 if rng.uniform() < refr_frac else float(rng.choice([0.6, 0.8, 1.0]))
        sph[i]["material"] = R.make_material(
            op, float(rng.uniform(0, 1)), rng.uniform(0, 1, 3), rng.uniform(0, 1, 3),
            float(rng.choice([1.0, 1.33, 1.55, 2.4])))
    lg = np.zeros(m, R.LIGHT_DTYPE)
    for l in range(m):
        lg[l]["pos"] = [rng.uniform(-60, 60), rng.uniform(-20, 80), rng.uniform(-40, 90)]
        lg[l]["col"] = rng.uniform(0.2, 1, 3)
    return sph, lg


def test_random_bvh_scenes_vs_oracle(R, oracle, torch_cuda):
    """BVH scenes (65..400 spheres) against the oracle: clustered, overlapping
    and refractive spheres under several lights, so the device-only list
    paths (blocked_cap, closest_enter_list, container_list, their paired
    record loads and padding records) and their BVH fallbacks all run."""
    torch = torch_cuda
    rng = np.random.default_rng(4242)
    ctx = R.Context(0)
    for trial in range(10):
        n, m = int(rng.integers(65, 401)), int(rng.integers(1, 5))
        S = int(rng.choice([3, 6, 8, 10]))
        W, H = int(rng.integers(24, 72)), int(rng.integers(16, 48))
        aa = float(rng.choice([1.0, 3.0]))
        sph, lg = clustered_scene(rng, n, m)
        want = oracle.render(sph, lg, W, H, S, aa=aa)
        ctx.set_scene(sph, lg)
        assert ctx.scene_stats()["bvh_nodes"] > 0, (trial, n)
        out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        ctx.render_device(W, H, out.data_ptr(), alias_factor=aa, stack_size=S,
                          stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert bits_equal(got, want), (trial, n, m, S, W, H, aa, first_mismatch(got, want))
    ctx.close()


def test_large_scene_global_material_path(R, oracle):
    """n + 1 > 1025 materials: the kernel reads materials from global memory."""
    rng = np.random.default_rng(99)
    sph, lg = random_scene(rng, 1100, 2)
    sph["radius"] *= 0.3
    want = oracle.render(sph, lg, 24, 14, 4)
    got = R.render(sph, lg, 24, 14, stack_size=4)
    assert bits_equal(got, want), first_mismatch(got, want)


def test_sharded_render_assembles_to_full_frame(R, golden, torch_cuda):
    """Row-cyclic shards (rtg_render_device) + dist.assemble == 1-GPU frame."""
    from rtg_amd import dist
    torch = torch_cuda
    c = golden["configs"]["c2"]
    sph, lg = load_scene("c2", c["spheres"], c["lights"])
    W, H, S, B = c["W"], c["H"], c["stack_size"], 16
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    for G in (1, 3, 8):
        Rmax = dist.padded_rows(H, B, G)
        buf = torch.zeros((G, Rmax, W, 3), dtype=torch.float32, device="cuda")
        stream = torch.cuda.current_stream().cuda_stream
        for g in range(G):
            ctx.render_device(W, H, buf[g].data_ptr(), stack_size=S, row_block=B, shard=g,
                              n_shards=G, stream=stream)
        torch.cuda.synchronize()
        fb = dist.assemble(buf, H, B).cpu().numpy()
        assert canon_md5(fb) == c["fb_md5"], G
        # the native assemble kernel (rtg_assemble_shards_device)
        frame = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        ctx.assemble_shards_device(buf.data_ptr(), G, Rmax, W, H, B, frame.data_ptr(), stream)
        torch.cuda.synchronize()
        assert canon_md5(frame.cpu().numpy()) == c["fb_md5"], G
        # the peer-copy ablation's placement (rtg_place_shard_device): every
        # shard straight into its rows of the frame, no gather buffer
        frame.fill_(7.0)
        for g in range(G):
            ctx.place_shard_device(buf[g].data_ptr(), g, G, W, H, B, frame.data_ptr(), stream)
        torch.cuda.synchronize()
        assert canon_md5(frame.cpu().numpy()) == c["fb_md5"], ("place", G)
    # odd widths take the 4-byte copy path; 16-byte path for W % 4 == 0
    for (W2, H2, G, B2) in [(37, 29, 3, 4), (64, 33, 5, 8), (1, 7, 2, 1)]:
        Rmax = dist.padded_rows(H2, B2, G)
        buf = torch.randn((G, Rmax, W2, 3), dtype=torch.float32, device="cuda")
        frame = torch.empty((H2, W2, 3), dtype=torch.float32, device="cuda")
        ctx.assemble_shards_device(buf.data_ptr(), G, Rmax, W2, H2, B2, frame.data_ptr(), 0)
        torch.cuda.synchronize()
        want = dist.assemble(buf.cpu().numpy(), H2, B2)
        assert np.array_equal(frame.cpu().numpy(), want), (W2, H2, G, B2)
        frame.fill_(-1.0)
        for g in range(G):
            ctx.place_shard_device(buf[g].data_ptr(), g, G, W2, H2, B2, frame.data_ptr(), 0)
        torch.cuda.synchronize()
        assert np.array_equal(frame.cpu().numpy(), want), ("place", W2, H2, G, B2)
    ctx.close()


def test_launch_order_feedback_keeps_frames(R, golden, torch_cuda):
    """Launch-order feedback (cull_groups_kernel: groups listed by the previous
    launch's measured times) only reorders work: repeated renders of one
    geometry, more geometries than the context keeps (least recently used
    entries replaced), row-list renders, a scene change and the flag that
    turns it off all give the golden frame."""
    from rtg_amd import dist
    torch = torch_cuda
    c = golden["configs"]["c2"]
    sph, lg = load_scene("c2", c["spheres"], c["lights"])
    W, H, S, B = c["W"], c["H"], c["stack_size"], 8
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    stream = torch.cuda.current_stream().cuda_stream
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    for flags in (0, ctx.LAUNCH_NO_ORDER_FEEDBACK, 0):
        ctx.set_variant(0, flags)
        for _ in range(3):
            out.fill_(5.0)
            ctx.render_device(W, H, out.data_ptr(), stack_size=S, stream=stream)
            torch.cuda.synchronize()
            assert canon_md5(out.cpu().numpy()) == c["fb_md5"], flags
    ctx.set_variant(0, 0)
    G = 12  # 12 shard geometries > the 8 kept: two passes replace entries
    Rmax = dist.padded_rows(H, B, G)
    buf = torch.zeros((G, Rmax, W, 3), dtype=torch.float32, device="cuda")
    for _ in range(2):
        for g in range(G):
            ctx.render_device(W, H, buf[g].data_ptr(), stack_size=S, row_block=B, shard=g,
                              n_shards=G, stream=stream)
        torch.cuda.synchronize()
        assert canon_md5(dist.assemble(buf, H, B).cpu().numpy()) == c["fb_md5"]
    rows = torch.arange(H - 1, -1, -1, dtype=torch.int32, device="cuda")  # bottom up
    for _ in range(2):
        out.fill_(5.0)
        ctx.render_rows_device(W, H, rows.data_ptr(), H, out.data_ptr(), stack_size=S,
                               stream=stream)
        torch.cuda.synchronize()
        assert canon_md5(out.flip(0).cpu().numpy()) == c["fb_md5"]
    # two streams rendering the same geometry at once share its cost table
    # (a race on a scheduling hint only)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out2 = torch.empty_like(out)
    for _ in range(3):
        out.fill_(5.0)
        out2.fill_(5.0)
        torch.cuda.synchronize()  # the fills (current stream) before s1 / s2 render
        ctx.render_device(W, H, out.data_ptr(), stack_size=S, stream=s1.cuda_stream)
        ctx.render_device(W, H, out2.data_ptr(), stack_size=S, stream=s2.cuda_stream)
        torch.cuda.synchronize()
        assert canon_md5(out.cpu().numpy()) == c["fb_md5"]
        assert canon_md5(out2.cpu().numpy()) == c["fb_md5"]
    c3 = golden["configs"]["c1"]  # another scene, then back
    sph3, lg3 = load_scene("c1", c3["spheres"], c3["lights"])
    ctx.set_scene(sph3, lg3)
    small = torch.empty((c3["H"], c3["W"], 3), dtype=torch.float32, device="cuda")
    for _ in range(2):
        ctx.render_device(c3["W"], c3["H"], small.data_ptr(), stack_size=c3["stack_size"],
                          stream=stream)
        torch.cuda.synchronize()
        assert canon_md5(small.cpu().numpy()) == c3["fb_md5"]
    ctx.set_scene(sph, lg)
    for _ in range(2):
        ctx.render_device(W, H, out.data_ptr(), stack_size=S, stream=stream)
        torch.cuda.synchronize()
        assert canon_md5(out.cpu().numpy()) == c["fb_md5"]
    ctx.close()


def test_failed_launch_leaves_slots_consistent(R, golden, torch_cuda):
    """A render that fails after the launch scratch is chosen (the counting
    build has no kernel for a maskless compacted scene: an empty scene) leaves
    the slot ring and the cost entries as the last good launch left them, so
    more good renders than the ring holds (rtg_context::kSlots = 4) still give
    the golden frame (the counter set a slot's next cull pass adds
    to must have been zeroed by a trace kernel)."""
    torch = torch_cuda
    c = golden["configs"]["c2"]
    sph, lg = load_scene("c2", c["spheres"], c["lights"])
    W, H, S = c["W"], c["H"], c["stack_size"]
    ctx = R.Context(0)
    stream = torch.cuda.current_stream().cuda_stream
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")

    def good(k):
        for _ in range(k):
            out.fill_(5.0)
            ctx.render_device(W, H, out.data_ptr(), stack_size=S, stream=stream)
            torch.cuda.synchronize()
            assert canon_md5(out.cpu().numpy()) == c["fb_md5"]

    ctx.set_scene(sph, lg)
    good(2)
    ctx.set_scene(sph[:0], lg)  # no spheres: compacted, no masks
    ctx.set_variant(120)
    for _ in range(3):
        with pytest.raises(R.RtgError):
            ctx.render_device(W, H, out.data_ptr(), stack_size=S, stream=stream)
    ctx.set_variant(0)
    ctx.set_scene(sph, lg)
    good(9)
    ctx.close()


@pytest.mark.parametrize("name", ["c2", "c1"])
def test_group_list_partitions(R, golden, torch_cuda, name):
    """The compacted launch's list (cull_groups_kernel: kListParts partitions,
    each with its own run counters; four runs for a whole C2 frame, eight for
    C1's short launch): over a cold launch, a launch whose cull pass sums the
    cost table and a launch ordered by it, every listed group appears once, has
    a non-empty sphere mask, and every group with a non-zero pixel is listed
    (the others were zero-filled by the cull pass)."""
    torch = torch_cuda
    c = golden["configs"][name]
    sph, lg = load_scene(name, c["spheres"], c["lights"])
    W, H, S = c["W"], c["H"], c["stack_size"]
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    stream = torch.cuda.current_stream().cuda_stream
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    ppw = 64 // 9
    groups = (W * H + ppw - 1) // ppw
    for launch in range(3):
        out.fill_(5.0)
        ctx.render_device(W, H, out.data_ptr(), stack_size=S, stream=stream)
        torch.cuda.synchronize()
        assert canon_md5(out.cpu().numpy()) == c["fb_md5"]
        d = ctx.diag_group_list()
        lst = d["list"].astype(np.int64)
        assert len(lst) == int(d["runs"].sum()) > 0
        assert len(np.unique(lst)) == len(lst) and lst.max() < groups
        assert (d["sel"] != 0).all()
        px = (out.cpu().numpy().reshape(-1, 3) != 0).any(axis=1)
        lit = np.unique(np.nonzero(px)[0] // ppw)
        assert np.isin(lit, lst).all(), launch
    ctx.close()


@pytest.mark.parametrize("variant", [0, 9])
def test_variant_full_frames(R, golden, torch_cuda, variant):
    """Kernel mappings over whole frames, sharded frames, row lists and
    back-to-back launches on two streams."""
    from rtg_amd import dist
    torch = torch_cuda
    ctx = R.Context(0)
    ctx.set_variant(variant)
    for name in ["c1", "c3"]:
        c = golden["configs"][name]
        sph, lg = load_scene(name, c["spheres"], c["lights"])
        W, H, S = c["W"], c["H"], c["stack_size"]
        ctx.set_scene(sph, lg)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        a = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        b = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        for _ in range(2):
            ctx.render_device(W, H, a.data_ptr(), stack_size=S, stream=s1.cuda_stream)
            ctx.render_device(W, H, b.data_ptr(), stack_size=S, stream=s2.cuda_stream)
        torch.cuda.synchronize()
        assert canon_md5(a.cpu().numpy()) == c["fb_md5"], name
        assert canon_md5(b.cpu().numpy()) == c["fb_md5"], name
    c = golden["configs"]["c2"]
    sph, lg = load_scene("c2", c["spheres"], c["lights"])
    W, H, S, B, G = c["W"], c["H"], c["stack_size"], 16, 3
    ctx.set_scene(sph, lg)
    Rmax = dist.padded_rows(H, B, G)
    buf = torch.zeros((G, Rmax, W, 3), dtype=torch.float32, device="cuda")
    stream = torch.cuda.current_stream().cuda_stream
    for g in range(G):
        rows = torch.tensor(R.shard_row_indices(H, B, g, G), dtype=torch.int32, device="cuda")
        ctx.render_rows_device(W, H, rows.data_ptr(), rows.numel(), buf[g].data_ptr(),
                               stack_size=S, stream=stream)
    torch.cuda.synchronize()
    fb = dist.assemble(buf, H, B).cpu().numpy()
    assert canon_md5(fb) == c["fb_md5"]
    ctx.close()


def test_device_max_and_ppm_bytes(R, golden, torch_cuda):
    torch = torch_cuda
    c = golden["configs"]["ref800"]
    sph, lg = load_scene("ref800", c["spheres"], c["lights"])
    W, H = c["W"], c["H"]
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    fb = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    mx = torch.empty(1, dtype=torch.float32, device="cuda")
    out = torch.empty(H * W * 3, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    ctx.render_device(W, H, fb.data_ptr(), stack_size=c["stack_size"], stream=s)
    ctx.max_colour_device(fb.data_ptr(), W * H, mx.data_ptr(), stream=s)
    ctx.ppm_bytes_device(fb.data_ptr(), W * H, mx.data_ptr(), out.data_ptr(), stream=s)
    torch.cuda.synchronize()
    assert np.float32(mx.item()).view(np.uint32) == c["max_colour_bits"]
    data = b"P6\n%d %d\n255\n" % (W, H) + out.cpu().numpy().tobytes()
    assert md5(data) == c["ppm_md5"]
    # all-black frame: max -> 1 (algebra.h:86-88)
    z = torch.zeros((4, 4, 3), dtype=torch.float32, device="cuda")
    ctx.max_colour_device(z.data_ptr(), 16, mx.data_ptr(), stream=s)
    torch.cuda.synchronize()
    assert mx.item() == 1.0
    ctx.close()


def test_errors_are_returned_not_fatal(R):
    sph, lg = R.reference_scene()
    with pytest.raises(R.RtgError):
        R.render(sph, lg, 8, 8, stack_size=0)
    with pytest.raises(R.RtgError):
        R.render(sph, lg, 8, 8, stack_size=17)
    with pytest.raises(R.RtgError):
        R.render(sph, lg, 8, 8, device=64)
    with pytest.raises(R.RtgError):
        R.render_rows(sph, lg, 8, 8, [8])
    # scenes of RTG_MAX_SPHERES (2^22) spheres or more are rejected before the
    # sphere array is read (the kernel's 22-bit index fields, 32-bit offsets)
    ctx = R.Context(0)
    one = np.zeros(1, R.SPHERE_DTYPE)
    rc = R.lib().rtg_context_set_scene(ctx._h, ctypes.c_void_p(one.ctypes.data), 1 << 22, None, 0)
    assert rc == -1 and b"spheres" in R.lib().rtg_last_error()
    ctx.close()
    # still usable afterwards
    fb = R.render(sph, lg, 8, 8)
    assert fb.shape == (8, 8, 3)


def _variant_small_frames(R, golden, torch, variant, names=("ref800", "c2", "c3", "c5")):
    ctx = R.Context(0)
    ctx.set_variant(variant)
    for name in names:
        c = golden["configs"][name]
        sph, lg = load_scene(name, c["spheres"], c["lights"])
        sw, sh = c["small"]["W"], c["small"]["H"]
        want = load_f32(os.path.join(GOLDEN, f"{name}.small.f32"), (sh, sw, 3))
        ctx.set_scene(sph, lg)
        out = torch.empty((sh, sw, 3), dtype=torch.float32, device="cuda")
        ctx.render_device(sw, sh, out.data_ptr(), stack_size=c["stack_size"],
                          stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert bits_equal(got, want), (name, variant, first_mismatch(got, want))
    ctx.close()


@pytest.mark.parametrize("variant", SHIPPED)
def test_kernel_variants_small_frames(R, golden, torch_cuda, variant):
    """Every shipped kernel variant (rtg_launch_opts.variant) is bit-exact
    too.  The probe build 110 has no BVH instantiation: on a BVH scene it
    returns an error instead of a frame."""
    if variant == 110:
        _variant_small_frames(R, golden, torch_cuda, variant, ("ref800", "c2", "c3"))
        c = golden["configs"]["c5"]
        sph, lg = load_scene("c5", c["spheres"], c["lights"])
        ctx = R.Context(0)
        ctx.set_variant(110)
        ctx.set_scene(sph, lg)
        out = torch_cuda.empty((8, 8, 3), dtype=torch_cuda.float32, device="cuda")
        with pytest.raises(R.RtgError):
            ctx.render_device(8, 8, out.data_ptr(), stack_size=c["stack_size"])
        ctx.close()
    else:
        _variant_small_frames(R, golden, torch_cuda, variant)


def test_ab_variants(R, golden, oracle, torch_cuda):
    """The A/B kernel variants (measured, not adopted) of a `make AB=1`
    library: small frames and random scenes.  The shipped library leaves them
    out, and rejects them."""
    ctx = R.Context(0)
    built = []
    for v in AB_VARIANTS:
        try:
            ctx.set_variant(v)
            built.append(v)
        except R.RtgError:
            pass
    ctx.close()
    if not built:
        pytest.skip("A/B variants not built (make AB=1)")
    for v in built:
        _variant_small_frames(R, golden, torch_cuda, v)
        _random_vs_oracle(R, oracle, torch_cuda, v, trials=6)


def test_counting_build(R, golden, torch_cuda):
    """The executed-work counting build (variant 120, rtg_diag_counts): the
    same frame bit for bit, and its lane-level counts of the per-lane
    algorithm units equal the host build's (tests/golden/unit_counts.json);
    wave-level counts bound lane-level ones (at most 64 lanes per wave)."""
    import json
    torch = torch_cuda
    fix = json.load(open(os.path.join(GOLDEN, "unit_counts.json")))
    ctx = R.Context(0)
    ctx.set_variant(120)
    for name, want in fix["frames"].items():
        c = golden["configs"][name]
        sph, lg = load_scene(name, c["spheres"], c["lights"])
        sw, sh = c["small"]["W"], c["small"]["H"]
        ctx.set_scene(sph, lg)
        ctx.diag_counts(reset=True)
        out = torch.empty((sh, sw, 3), dtype=torch.float32, device="cuda")
        ctx.render_device(sw, sh, out.data_ptr(), stack_size=c["stack_size"],
                          stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ref = load_f32(os.path.join(GOLDEN, f"{name}.small.f32"), (sh, sw, 3))
        assert bits_equal(out.cpu().numpy(), ref), name
        wv, lv = ctx.diag_counts(reset=True)
        got = {u: int(lv[R.UNIT_NAMES.index(u)]) for u in fix["units"]}
        assert got == want, (name, got, want)
        u = np.array([nm.startswith("U.") for nm in R.UNIT_NAMES])  # 1 per lane and execution
        assert (wv[u] <= lv[u]).all() and (lv[u] <= 64 * wv[u]).all(), name
        k = R.UNIT_NAMES.index("U.sample")
        assert 0 < lv[k] <= sw * sh * 9 and wv[k] > 0, name
    # a BVH scene (C5, n > 64) runs its own counting instantiation
    c = golden["configs"]["c5"]
    sph, lg = load_scene("c5", c["spheres"], c["lights"])
    ctx.set_scene(sph, lg)
    out = torch.empty((54, 96, 3), dtype=torch.float32, device="cuda")
    ctx.render_device(96, 54, out.data_ptr(), stack_size=c["stack_size"])
    torch.cuda.synchronize()
    assert bits_equal(out.cpu().numpy(), load_f32(os.path.join(GOLDEN, "c5.small.f32"), (54, 96, 3)))
    wv, lv = ctx.diag_counts(reset=True)
    assert wv[R.UNIT_NAMES.index("U.bvhNode")] > 0 and wv[R.UNIT_NAMES.index("U.bvhSlot")] > 0
    ctx.close()


@pytest.mark.parametrize("variant", [9, 0])
def test_wave_timeline_diagnostic(R, golden, torch_cuda, variant):
    """RTG_LAUNCH_TIMELINE: one record per wave, output unchanged."""
    torch = torch_cuda
    c = golden["configs"]["c2"]
    sph, lg = load_scene("c2", c["spheres"], c["lights"])
    W, H, S = c["W"], c["H"], c["stack_size"]
    ctx = R.Context(0)
    ctx.set_scene(sph, lg)
    ctx.set_variant(variant, ctx.LAUNCH_TIMELINE)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    ctx.render_device(W, H, out.data_ptr(), stack_size=S,
                      stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert canon_md5(out.cpu().numpy()) == c["fb_md5"]
    rec = ctx.diag_timeline()
    groups = -(-(W * H) // 7)
    if variant == 9:
        assert len(rec) == ((W + 15) // 16) * ((H + 15) // 16) * 4
    else:  # compacted launch: about one wave per listed group
        assert 0 < len(rec) <= groups
        pc, grp = (rec[:, 3] >> 4) & 127, rec[:, 3] >> 11  # tag: first group's mask, index
        assert pc.max() >= 1 and (pc <= c["spheres"]).all() and (grp < groups).all()
    dur = (rec[:, 1].astype(np.int64) - rec[:, 0].astype(np.int64)) % (1 << 32)
    assert (dur < 100_000_000).all()  # < 1 s each
    ctx.close()


def _render_multi_checks(R, golden, devs):
    c = golden["configs"]["c2"]
    sph, lg = load_scene("c2", c["spheres"], c["lights"])
    n = R.device_count()
    for B in (16, 8):
        fb, tm = R.render_multi(sph, lg, c["W"], c["H"], devices=devs, stack_size=c["stack_size"],
                                row_block=B)
        assert canon_md5(fb) == c["fb_md5"], (devs, B)
        assert tm[0] > 0 and tm[2] >= tm[0]
    # persistent handle: several frames and sizes, one communicator
    mc = R.MultiContext(devs)
    mc.set_scene(sph, lg)
    for _ in range(2):
        fb, tm = mc.render(c["W"], c["H"], stack_size=c["stack_size"])
        assert canon_md5(fb) == c["fb_md5"]
    small, _ = mc.render(40, 30, stack_size=c["stack_size"])
    assert bits_equal(small, R.render(sph, lg, 40, 30, stack_size=c["stack_size"]))
    # the peer-copy ablation (no collective, no assemble pass)
    mc.set_gather(mc.GATHER_PEER_COPY)
    for B in (16, 8, 7):
        fb, tm = mc.render(c["W"], c["H"], stack_size=c["stack_size"], row_block=B)
        assert canon_md5(fb) == c["fb_md5"], ("peer", devs, B)
    mc.set_gather(mc.GATHER_RCCL)
    fb, _ = mc.render(c["W"], c["H"], stack_size=c["stack_size"])
    assert canon_md5(fb) == c["fb_md5"]
    with pytest.raises(R.RtgError):
        mc.set_gather(5)
    mc.close()
    with pytest.raises(R.RtgError):
        R.render_multi(sph, lg, 8, 8, devices=[0, 0])
    with pytest.raises(R.RtgError):
        R.render_multi(sph, lg, 8, 8, devices=[n + 3])


def test_render_multi_one_device(R, golden):
    """rtg_render_multi (one process, RCCL gather) with one device: the
    communicator has size 1, so this covers the render/gather/assemble code
    path but not a multi-rank gather."""
    _render_multi_checks(R, golden, [0])


def test_render_multi_several_devices(R, golden):
    """The same over every visible device (up to 8): the real multi-rank
    ncclGather.  Skipped, visibly, on a box with fewer than two GPUs."""
    n = R.device_count()
    if n < 2:
        pytest.skip(f"multi-device RCCL gather needs >= 2 GPUs ({n} visible): unverified here")
    _render_multi_checks(R, golden, list(range(min(n, 8))))


def test_unknown_variant_is_rejected(R, torch_cuda):
    """rtg_set_launch_opts accepts only the variants of the kernel table; the
    OpenCL-semantics variants (50, 59) change results and are reachable only
    through rtg_context_set_semantics."""
    ctx = R.Context(0)
    for bad in (7, 10, 13, 27, 50, 59, 101, 105, 109, -1, 1 << 20):
        with pytest.raises(R.RtgError):
            ctx.set_variant(bad)
    with pytest.raises(R.RtgError):
        ctx.set_variant(0, 0x100)  # unknown flag bit
    # the context still renders with its previous (default) variant
    sph, lg = R.reference_scene()
    ctx.set_scene(sph, lg)
    out = torch_cuda.empty((12, 16, 3), dtype=torch_cuda.float32, device="cuda")
    ctx.render_device(16, 12, out.data_ptr())
    torch_cuda.cuda.synchronize()
    assert bits_equal(out.cpu().numpy(), R.render(sph, lg, 16, 12))
    ctx.close()
    old = os.environ.get("RTG_VARIANT")
    try:
        for bad in ("7", "50", "x", ""):
            os.environ["RTG_VARIANT"] = bad
            with pytest.raises(R.RtgError):
                R.Context(0)
        os.environ["RTG_VARIANT"] = "9"
        R.Context(0).close()
    finally:
        if old is None:
            os.environ.pop("RTG_VARIANT", None)
        else:
            os.environ["RTG_VARIANT"] = old


def test_current_device_is_restored(R, golden, torch_cuda):
    """ABI calls select their context's device and restore the caller's
    current device on return (checked on the last visible device when there
    are several)."""
    torch = torch_cuda
    n = R.device_count()
    cur = n - 1
    torch.cuda.set_device(cur)
    try:
        sph, lg = R.reference_scene()
        R.render(sph, lg, 8, 6, device=0)
        assert torch.cuda.current_device() == cur
        R.render_multi(sph, lg, 8, 6, devices=list(range(min(n, 8))))
        assert torch.cuda.current_device() == cur
        ctx = R.Context(0)
        ctx.set_scene(sph, lg)
        assert torch.cuda.current_device() == cur
        ctx.close()
        assert torch.cuda.current_device() == cur
    finally:
        torch.cuda.set_device(0)


@pytest.mark.parametrize("extra", [[], ["--gpus", "1"]])
def test_host_driver_scene_file_ppm(R, golden, tmp_path, extra):
    """The C++ host driver (the reference's main() flow) on the reference scene
    file writes the reference's PPM byte for byte, single- or multi-GPU path."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "raytracer-gamma_amd", "rtg_main")
    scene = os.path.join(root, "scenes", "reference.scene")
    out = str(tmp_path / "o.ppm")
    r = subprocess.run([exe, "--scene", scene, "--out", out] + extra, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert md5(open(out, "rb").read()) == golden["configs"]["ref800"]["ppm_md5"]


def test_opencl_semantics_vs_oracle(R, oracle, torch_cuda):
    """rtg_context_set_semantics(RTG_SEMANTICS_OPENCL): the reference OpenCL
    kernel's semantics, bit-exact against the OpenCL-semantics oracle, through
    the sample kernel and its nAA > 8 fallback."""
    torch = torch_cuda
    ctx = R.Context(0)
    ctx.set_semantics(ctx.SEMANTICS_OPENCL)
    rng = np.random.default_rng(2027)
    cases = [(5, 3.0, -4.0, None)] + [None] * 14
    for trial, case in enumerate(cases):
        if case is None:
            S = int(rng.integers(1, 17))
            aa = float(rng.choice([1.0, 2.0, 3.0, 9.0]))
            zoom = float(rng.choice([-4.0, 3.0]))
            n, m = int(rng.integers(0, 20)), int(rng.integers(0, 5))
            sph, lg = random_scene(rng, n, m)
            if zoom > 0:
                sph["pos"][:, 2] *= -1.0
            W, H = int(rng.integers(1, 60)), int(rng.integers(1, 40))
        else:
            S, aa, zoom, _ = case
            sph, lg = R.reference_scene()
            W, H = 160, 120
        want = oracle.render_cl(sph, lg, W, H, S, aa=aa, zoom=zoom)
        ctx.set_scene(sph, lg)
        out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
        ctx.render_device(W, H, out.data_ptr(), zoom=zoom, alias_factor=aa, stack_size=S,
                          stream=torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        assert bits_equal(got, want), (trial, S, W, H, aa, first_mismatch(got, want))
    ctx.set_semantics(ctx.SEMANTICS_CPU)
    sph, lg = R.reference_scene()
    ctx.set_scene(sph, lg)
    out = torch.empty((60, 80, 3), dtype=torch.float32, device="cuda")
    ctx.render_device(80, 60, out.data_ptr(), stack_size=5)
    torch.cuda.synchronize()
    assert bits_equal(out.cpu().numpy(), oracle.render(sph, lg, 80, 60, 5))
    with pytest.raises(R.RtgError):
        ctx.set_semantics(7)
    ctx.close()


def test_opencl_reference_kernel_pins_oracle(R, oracle, torch_cuda):
    """The reference's OWN OpenCL kernel (raytrace_kernel.cl:870-973, compiled
    for gfx950 in place from /root/reference by oracle/build_ref_cl.sh with
    correctly rounded division/sqrt and no contraction, launched as a HIP
    module: tests/clref.py) against the OpenCL-semantics oracle
    (oracle_render_rows_cl) and the kernel's kCL mode (variant 50 and its
    nAA > 8 fallback 59), bit for bit: the main.cpp scene and seeded random
    scenes of up to 20 spheres, several sizes, aliasFactors and zooms."""
    import clref
    torch = torch_cuda
    if not os.path.exists(clref.HSACO):
        pytest.skip("oracle/_ref/rtg_ref_cl.hsaco not built (needs /root/reference at build)")
    ref = clref.RefCL()
    ctx = R.Context(0)
    ctx.set_semantics(ctx.SEMANTICS_OPENCL)
    rng = np.random.default_rng(5150)
    cases = [(3.0, -4.0, None, 160, 120)] + [None] * 15
    try:
        for trial, case in enumerate(cases):
            if case is None:
                aa = float(rng.choice([1.0, 2.0, 3.0, 9.0]))
                zoom = float(rng.choice([-4.0, 3.0]))
                n, m = int(rng.integers(0, 21)), int(rng.integers(0, 5))
                sph, lg = random_scene(rng, n, m)
                if zoom > 0:
                    sph["pos"][:, 2] *= -1.0
                W, H = int(rng.integers(1, 64)), int(rng.integers(1, 40))
            else:
                aa, zoom, _, W, H = case
                sph, lg = R.reference_scene()
            want = ref.render(torch, sph, lg, W, H, zoom=zoom, aa=aa)
            orc = oracle.render_cl(sph, lg, W, H, 5, aa=aa, zoom=zoom)
            assert bits_equal(orc, want), (trial, W, H, aa, first_mismatch(orc, want))
            ctx.set_scene(sph, lg)
            out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
            ctx.render_device(W, H, out.data_ptr(), zoom=zoom, alias_factor=aa, stack_size=5,
                              stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            got = out.cpu().numpy()
            assert bits_equal(got, want), (trial, W, H, aa, first_mismatch(got, want))
    finally:
        ctx.close()
        ref.close()


def test_host_driver_opencl_semantics_ppm(R, oracle, tmp_path):
    """rtg_main --semantics opencl --depth 4 (the .cl's stack of 5): its PPM is
    the OpenCL-semantics oracle's PPM byte for byte."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "raytracer-gamma_amd", "rtg_main")
    out = str(tmp_path / "cl.ppm")
    r = subprocess.run([exe, "--semantics", "opencl", "--depth", "4", "--width", "200",
                        "--height", "150", "--out", out], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    sph, lg = R.reference_scene()
    want = R.ppm_file_bytes(oracle.render_cl(sph, lg, 200, 150, 5))
    assert open(out, "rb").read() == want


def test_fast_sqrt_rcp_exhaustive():
    """rtg_trace.h's short sequences for the correctly rounded square root and
    reciprocal (sqrt_rn / rcp_rn, used by every vnorm and every query's 1/2a)
    against the compiler's correctly rounded sqrtf and 1.f / x, and against an
    exact f64 rounding criterion, for EVERY binary32 bit pattern, on the GPU
    (tests/fpcheck/fpcheck_gpu.hip)."""
    so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fpcheck", "libfpcheck_gpu.so")
    L = ctypes.CDLL(so)
    out = (ctypes.c_ulonglong * 8)()
    assert L.fpcheck_run(ctypes.c_ulonglong(0), out) == 0
    sqrt_in, sqrt_lib, sqrt_exact, sqrt_all, rcp_in, rcp_lib, rcp_exact, rcp_all = list(out)
    # the fast ranges: [2^-96, FLT_MAX] and [2^-125, 2^125]
    assert sqrt_in == 0x7F7FFFFF - 0x0F800000 + 1
    assert rcp_in == 0x7E000000 - 0x01000000 + 1
    assert (sqrt_lib, sqrt_exact, sqrt_all) == (0, 0, 0), list(out)
    assert (rcp_lib, rcp_exact, rcp_all) == (0, 0, 0), list(out)


def test_fast_f64_islands():
    """rtg_trace.h's trimmed f64 square root and quotient of the refraction
    (sqrt_d_unit for sinA1 = sqrt(1 - cos^2), raytracer.h:683, and
    div_d_fresnel for polarisedReflection's quotient, raytracer.h:388-393)
    against sqrt() and the IEEE division bit for bit on the GPU: every float
    cosine in [0, 1) and 2^32 random Fresnel operand pairs
    (tests/fpcheck/fpcheck_gpu.hip)."""
    so = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fpcheck", "libfpcheck_gpu.so")
    L = ctypes.CDLL(so)
    out = (ctypes.c_ulonglong * 4)()
    assert L.fpcheck_f64_run(ctypes.c_ulonglong(0), out) == 0
    sqrt_in, sqrt_bad, div_in, div_bad = list(out)
    assert sqrt_in == 0x3F800000
    assert div_in > 3 * 10**9, list(out)
    assert (sqrt_bad, div_bad) == (0, 0), list(out)
