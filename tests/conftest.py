"""Shared fixtures for the rtg test-suite.

Markers: `gpu` — needs an MI355X (run on the GPU box with `-m gpu`); everything
else runs on the CPU-only container.

The oracle (oracle/, C restatement of the reference) is TEST INFRASTRUCTURE:
it is loaded here only as the checker.
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "raytracer-gamma_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
BUILD = os.path.join(ROOT, "tests", "_build")
# RTG_ASAN=1: load the AddressSanitizer/UBSan builds of the CPU checkers
# (tests/asan/Makefile; tests/test_sanitizers.py runs the suite that way).
ASAN = os.environ.get("RTG_ASAN") == "1"
ASAN_BUILD = os.path.join(BUILD, "asan")
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X)")


def _make(target_dir, *targets):
    subprocess.run(["make", "-s", "-C", target_dir, *targets], check=True)


@pytest.fixture(scope="session")
def rtg():
    if not os.path.exists(os.path.join(PKG, "librtg.so")):
        _make(PKG, "librtg.so")
    import rtg_amd
    return rtg_amd


class Oracle:
    """ctypes front of oracle/build/librtg_oracle.so (the checker)."""

    def __init__(self):
        path = os.path.join(ROOT, "oracle", "build", "librtg_oracle.so")
        if ASAN:
            path = os.path.join(ASAN_BUILD, "librtg_oracle.so")
        elif not os.path.exists(path):
            _make(os.path.join(ROOT, "oracle"), "build/librtg_oracle.so")
        self.lib = ctypes.CDLL(path)
        self.lib.oracle_max_colour.restype = ctypes.c_float
        self.lib.oracle_max_colour.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong]
        self.lib.oracle_ppm_bytes.argtypes = [ctypes.c_void_p, ctypes.c_ulonglong,
                                              ctypes.c_float, ctypes.c_void_p]

    def render(self, sph, lg, W, H, S, rows=None, aa=3.0, zoom=-4.0, threads=None):
        rows = np.arange(H, dtype=np.uint32) if rows is None else np.asarray(rows, np.uint32)
        out = np.zeros((len(rows), W, 3), np.float32)
        cnt = (ctypes.c_ulonglong * 3)()
        threads = threads or min(16, os.cpu_count() or 1)
        rc = self.lib.oracle_render_rows(P(sph), len(sph), P(lg), len(lg), W, H,
                                         ctypes.c_float(zoom), ctypes.c_float(aa), S, P(rows),
                                         len(rows), P(out), threads, cnt)
        assert rc == 0
        self.counters = [int(c) for c in cnt]
        return out

    def render_cl(self, sph, lg, W, H, S, rows=None, aa=3.0, zoom=-4.0, threads=None):
        """The reference OpenCL kernel's semantics (oracle_render_rows_cl)."""
        rows = np.arange(H, dtype=np.uint32) if rows is None else np.asarray(rows, np.uint32)
        out = np.zeros((len(rows), W, 3), np.float32)
        threads = threads or min(16, os.cpu_count() or 1)
        rc = self.lib.oracle_render_rows_cl(P(sph), len(sph), P(lg), len(lg), W, H,
                                            ctypes.c_float(zoom), ctypes.c_float(aa), S, P(rows),
                                            len(rows), P(out), threads)
        assert rc == 0
        return out

    def max_colour(self, fb):
        fb = np.ascontiguousarray(fb, np.float32)
        return self.lib.oracle_max_colour(P(fb), fb.size // 3)

    def ppm_bytes(self, fb, mx):
        fb = np.ascontiguousarray(fb, np.float32)
        out = np.empty(fb.size, np.uint8)
        self.lib.oracle_ppm_bytes(P(fb), fb.size // 3, ctypes.c_float(mx), P(out))
        return out


def P(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None and a.size else None


@pytest.fixture(scope="session")
def oracle():
    return Oracle()


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def load_scene(name, n, m):
    import rtg_amd
    raw = open(os.path.join(GOLDEN, f"{name}.scene.bin"), "rb").read()
    assert len(raw) == 48 * n + 24 * m
    sph = np.frombuffer(raw[:48 * n], rtg_amd.SPHERE_DTYPE).copy()
    lg = np.frombuffer(raw[48 * n:], rtg_amd.LIGHT_DTYPE).copy()
    return sph, lg


def load_f32(path, shape):
    return np.fromfile(path, np.float32).reshape(shape)


def md5(b):
    return hashlib.md5(b).hexdigest()


def canon(fb):
    """uint32 bits with every NaN as 0xFFC00000 (the x86 default NaN).  NaN
    payload/sign is implementation-defined (two x86 compilers of the reference
    source disagree on it), so parity = bit-exact non-NaN values + identical
    NaN positions."""
    fb = np.ascontiguousarray(fb, np.float32)
    b = fb.view(np.uint32).copy()
    b[np.isnan(fb)] = 0xFFC00000
    return b


def bits_equal(a, b):
    """Bit-exact equality of every non-NaN value, NaNs at the same places."""
    return a.shape == b.shape and bool((canon(a) == canon(b)).all())


def canon_md5(fb):
    return md5(canon(fb).tobytes())


def first_mismatch(a, b):
    d = np.argwhere(canon(a) != canon(b))
    if len(d) == 0:
        return None
    i = tuple(d[0])
    return f"{len(d)} words differ; first at {i}: {a[i]!r} vs {b[i]!r}"


def random_scene(rng, n, m):
    import rtg_amd as R
    sph = np.zeros(n, R.SPHERE_DTYPE)
    for i in range(n):
        sph[i]["pos"] = [rng.uniform(-12, 12), rng.uniform(-8, 8), rng.uniform(-40, -4)]
        sph[i]["radius"] = rng.uniform(0.5, 4.0)
        sph[i]["material"] = R.make_material(
            float(rng.choice([0.0, 0.2, 0.5, 0.8, 1.0])), float(rng.uniform(0, 1)),
            rng.uniform(0, 1, 3), rng.uniform(0, 1, 3), float(rng.choice([1.0, 1.33, 1.55, 2.4])))
    lg = np.zeros(m, R.LIGHT_DTYPE)
    for l in range(m):
        lg[l]["pos"] = [rng.uniform(-60, 60), rng.uniform(-20, 80), rng.uniform(-40, 90)]
        lg[l]["col"] = rng.uniform(0, 1, 3)
    return sph, lg
