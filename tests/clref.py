"""Test-only loader of the reference's own OpenCL kernel (raytrace_kernel.cl),
compiled for gfx950 by oracle/build_ref_cl.sh into oracle/_ref/rtg_ref_cl.hsaco
and launched as a HIP module through the process's HIP runtime (the one torch
loaded).  TEST INFRASTRUCTURE: it is the checker of the OpenCL-semantics
oracle and of the kernel's kCL mode, never part of the product path.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
HSACO = os.path.join(os.path.dirname(HERE), "oracle", "_ref", "rtg_ref_cl.hsaco")
KERNEL = b"rtg_ref_cl_raytrace"
LOCAL = 64  # the harness's reqd_work_group_size (ref_cl_harness.cl)


def _hip():
    """The HIP runtime already mapped into this process (torch's)."""
    path = None
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                path = line.split()[-1]
                break
    if path is None:
        raise RuntimeError("libamdhip64 not loaded (import torch and touch cuda first)")
    return ctypes.CDLL(path)


class RefCL:
    def __init__(self):
        if not os.path.exists(HSACO):
            raise FileNotFoundError(HSACO)
        self.L = _hip()
        self.mod = ctypes.c_void_p()
        self.fn = ctypes.c_void_p()
        self._ck(self.L.hipModuleLoad(ctypes.byref(self.mod), HSACO.encode()), "hipModuleLoad")
        self._ck(self.L.hipModuleGetFunction(ctypes.byref(self.fn), self.mod, KERNEL),
                 "hipModuleGetFunction")

    @staticmethod
    def _ck(rc, what):
        if rc != 0:
            raise RuntimeError(f"{what} failed: hipError {rc}")

    def render(self, torch, spheres, lights, W, H, zoom=-4.0, aa=3.0):
        """The reference kernel's frame (H, W, 3) float32 for one scene
        (spheres, lights <= 64 each: the kernel copies them one per work-item)."""
        n, m = len(spheres), len(lights)
        assert n <= LOCAL and m <= LOCAL, (n, m)
        total = W * H
        groups = (total + LOCAL - 1) // LOCAL
        dev = torch.device("cuda")
        sph = torch.from_numpy(np.frombuffer(spheres.tobytes(), np.uint8).copy()).to(dev) \
            if n else torch.zeros(48, dtype=torch.uint8, device=dev)
        lgt = torch.from_numpy(np.frombuffer(lights.tobytes(), np.uint8).copy()).to(dev) \
            if m else torch.zeros(24, dtype=torch.uint8, device=dev)
        # every work-item of the grid writes its pixel: pad to the grid
        dst = torch.full((groups * LOCAL * 3,), 7.0, dtype=torch.float32, device=dev)
        args = [ctypes.c_void_p(sph.data_ptr()), ctypes.c_uint(n),
                ctypes.c_void_p(lgt.data_ptr()), ctypes.c_uint(m),
                ctypes.c_uint(W), ctypes.c_uint(H), ctypes.c_float(zoom), ctypes.c_float(aa),
                ctypes.c_void_p(dst.data_ptr())]
        params = (ctypes.c_void_p * len(args))(*[ctypes.cast(ctypes.byref(a), ctypes.c_void_p)
                                                 for a in args])
        torch.cuda.synchronize()
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        self._ck(self.L.hipModuleLaunchKernel(self.fn, ctypes.c_uint(groups), ctypes.c_uint(1),
                                              ctypes.c_uint(1), ctypes.c_uint(LOCAL),
                                              ctypes.c_uint(1), ctypes.c_uint(1),
                                              ctypes.c_uint(0), stream, params, None),
                 "hipModuleLaunchKernel")
        torch.cuda.synchronize()
        return dst[:total * 3].cpu().numpy().reshape(H, W, 3)

    def close(self):
        if self.mod:
            self.L.hipModuleUnload(self.mod)
            self.mod = ctypes.c_void_p()
