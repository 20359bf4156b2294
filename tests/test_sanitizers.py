"""CPU checkers under AddressSanitizer + UBSan (SURVEY.md §5 "Race detection /
sanitizers").

tests/asan/Makefile builds oracle/rtg_oracle.c (the C restatement) and
tests/hostsim/hostsim.cpp (the kernel traversal and scene preparation of
rtg_trace.h / rtg_scene_pack.h, compiled for the host) with
-fsanitize=address,undefined -fno-sanitize-recover=all.  This test runs the
oracle and hostsim tests of tests/test_oracle.py in a child pytest with those
builds loaded (RTG_ASAN=1) and the ASan runtime preloaded: an out-of-bounds
access, use-after-free or undefined behaviour anywhere in them aborts the
child, and the test fails with its report.
"""
from __future__ import annotations

import os
import subprocess
import sys

from conftest import ROOT

# the oracle and kernel-traversal tests over every code path (flat, masked,
# BVH and list queries, edge cases, the OpenCL semantics); the slow
# full-frame, brute-force 1024-sphere and million-pair checks stay in the
# normal, unsanitised run (the whole CPU suite should take minutes)
SELECT = ("oracle_edge_cases or kernel_traversal_edge_cases or kernel_traversal_bvh_random or "
          "(kernel_traversal_random_scenes and v0) or (kernel_traversal_random_scenes and v9) or "
          "(oracle_small_frames and not c4 and not c5) or "
          "(kernel_traversal_small_frames and v0 and not c5) or "
          "(kernel_traversal_opencl_semantics)")


def test_oracle_and_hostsim_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "asan")], check=True)
    asan = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                          text=True, check=True).stdout.strip()
    env = dict(os.environ, RTG_ASAN="1", LD_PRELOAD=asan,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:halt_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        "-m", "not gpu", os.path.join(ROOT, "tests", "test_oracle.py"),
                        "-k", SELECT], cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=1500)
    tail = (r.stdout + r.stderr)[-6000:]
    assert r.returncode == 0, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error:" not in r.stderr, tail
    assert " passed" in r.stdout, tail
