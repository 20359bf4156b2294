"""CPU multi-process tests of the N > 1 path (gloo, world size 2 and 3).

Each rank renders its row-cyclic shard, rank 0 gathers the padded shard
buffers with ONE gather (the collective bench.py issues over RCCL on GPUs) and
restores row order with rtg_amd.dist.assemble; the result must equal the
1-rank frame bit for bit.  Shards are rendered here by the oracle (CPU
checker) with the global row list the C ABI's shard mapping gives, since there
is no GPU in this container.
"""
from __future__ import annotations

import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, B, S, result_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    sys.path.insert(0, os.path.join(ROOT, "raytracer-gamma_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import rtg_amd as R
    from rtg_amd import dist as rdist
    from conftest import Oracle
    orc = Oracle()
    sph, lg = R.generate_scene(8, 2, 42)
    Rmax = rdist.padded_rows(H, B, world)
    rows = R.shard_row_indices(H, B, rank, world)
    assert len(rows) == R.shard_rows(H, B, rank, world) <= Rmax
    buf = torch.zeros((Rmax, W, 3), dtype=torch.float32)
    if len(rows):
        buf[: len(rows)] = torch.from_numpy(orc.render(sph, lg, W, H, S, rows=rows, threads=2))
    gl = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gl, dst=0)
    if rank == 0:
        frame = rdist.assemble(torch.stack(gl), H, B).contiguous().numpy()
        np.save(result_path, frame)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,B", [(2, 48, 37, 4), (3, 40, 50, 8), (2, 32, 16, 16)])
def test_row_cyclic_gather_equals_single_rank(tmp_path, oracle, rtg, world, W, H, B):
    S = 4
    path = str(tmp_path / "frame.npy")
    mp.start_processes(_worker, args=(world, _free_port(), W, H, B, S, path), nprocs=world,
                       join=True, start_method="spawn")
    got = np.load(path)
    sph, lg = rtg.generate_scene(8, 2, 42)
    want = oracle.render(sph, lg, W, H, S)
    from conftest import bits_equal, first_mismatch
    assert bits_equal(got, want), first_mismatch(got, want)


def test_assemble_numpy_matches_torch(rtg):
    from rtg_amd import dist as rdist
    H, B, G, W = 45, 4, 3, 5
    Rmax = rdist.padded_rows(H, B, G)
    g = np.full((G, Rmax, W, 3), -1, np.float32)
    for s in range(G):
        rows = rtg.shard_row_indices(H, B, s, G)
        g[s, : len(rows)] = rows[:, None, None]
    a = rdist.assemble(g, H, B)
    t = rdist.assemble(torch.from_numpy(g), H, B).numpy()
    assert (a == t).all()
    assert (a[:, 0, 0] == np.arange(H)).all()


def test_chunk_bounds():
    """bench.py's chunks of a shard: whole row blocks, in order, covering the
    shard, each non-empty; with last_frac the last is about that share."""
    from rtg_amd import dist
    for nb in (1, 2, 3, 5, 34, 68, 135, 270):
        for K in (1, 2, 3, 4, 8):
            for f in (0.0, 0.15, 0.25, 0.5):
                b = dist.chunk_bounds(nb, K, 8, f)
                k = min(K, nb)
                assert len(b) == k + 1 and b[0] == 0 and b[-1] == 8 * nb, (nb, K, f, b)
                assert all(x % 8 == 0 for x in b)
                assert all(b[i + 1] > b[i] for i in range(k)), (nb, K, f, b)
                if f > 0 and k > 1 and nb >= 20:
                    assert abs((b[-1] - b[-2]) / (8 * nb) - f) <= 1.0 / nb, (nb, K, f, b)
    assert dist.default_chunks(8) == (3, 0.15) and dist.default_chunks(2) == (4, 0.15)
