"""GPU test of bench.py's N > 1 step (the driver's multi-GPU scaling run).

Two ranks share the box's one GPU and gather through host memory (gloo), so
the chunked pipeline the 8-GPU run uses — row-cyclic shards rendered in
chunks on two streams, each chunk gathered and put back in row order on rank
0's assembling stream — runs end to end on every GPU test pass, and its
fields are checked: the assembled frame is the golden frame, the per-rank
timings are non-negative and the rank-0 render + gather tail + assemble fit
in the step.
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench_lines(args, nproc, timeout=240):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py")] + args
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return lines[0]


@pytest.mark.parametrize("chunks", [0, 1])
def test_bench_two_rank_step(chunks):
    """bench.py --gpus 2 (gloo, both ranks on GPU 0) on C2: default chunking
    (4 chunks at two ranks) and a single gather."""
    out = _bench_lines(["--gpus", "2", "--steps", "4", "--warmup", "2", "--config", "c2",
                        "--dist-backend", "gloo", "--gather-chunks", str(chunks)], 2)
    assert out["n_gpus"] == 2
    assert out["parity"]["fb_md5_match"] is True
    assert out["parity"]["ppm_md5_match"] is True
    mg = out["multi_gpu"]
    assert mg["gather_chunks"] == (4 if chunks == 0 else 1)
    assert len(mg["render_ms_per_rank"]) == 2
    assert all(t > 0 for t in mg["render_ms_per_rank"])
    assert mg["gather_tail_ms_rank0"] >= 0.0
    assert mg["assemble_ms_rank0"] >= 0.0
    step = mg["step_ms"]
    assert mg["render_ms_per_rank"][0] + mg["gather_tail_ms_rank0"] + \
        mg["assemble_ms_rank0"] <= step * 1.05, mg
    assert out["value"] > 0 and abs(out["ms_per_step"] - step) < 1e-3 * step + 1e-3
