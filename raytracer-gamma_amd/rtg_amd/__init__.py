"""rtg_amd — ctypes binding of librtg.so, the MI355X raytracer-gamma hot path.

This is the binding a Python maintainer would add over the C ABI in
include/rtg.h (INTEGRATION.md shows the C/C++ and ctypes forms).  It mirrors
the reference's host interface for the path:

  reference                                   here
  ------------------------------------------  ------------------------------------
  struct Sphere / Light / Material (C)        SPHERE_DTYPE / LIGHT_DTYPE / MATERIAL_DTYPE
  setMatOpacity+setMatteGlossBalance+...      make_material()   (raytracer.h:53-74)
  scene of main.cpp:104-168                   generate_scene()  (+ SURVEY §8d generator)
  OpenCL raytrace kernel + enqueue/readback   render() / Context.render_device()
    (raytrace_kernel.cl:870, main.cpp:277-468)
  maxColourValuePixelBuffer (algebra.h:68)    max_colour_value()
  savePPM (main.cpp:43-91)                    save_ppm() / ppm_bytes()

There is no CPU fallback: every render call goes to the HIP kernel and raises
RtgError when the library or a GPU is missing.
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

# torch (when present) must own the HIP runtime of this process: librtg.so's
# libamdhip64.so.7 dependency then resolves to the runtime torch already
# loaded, so torch streams / pointers and ours are the same runtime's.
try:  # pragma: no cover - import side effect only
    import torch  # noqa: F401
except Exception:  # torch absent: librtg loads /opt/rocm's runtime itself
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# RTG_LIB: an alternative build of the same library (compiler-flag A/B runs).
LIB_PATH = os.environ.get("RTG_LIB") or os.path.join(os.path.dirname(_HERE), "librtg.so")

VEC_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("z", "<f4")])
MATERIAL_DTYPE = np.dtype([("matteColour", "<f4", 3), ("glossColour", "<f4", 3),
                           ("opacity", "<f4"), ("refractiveIndex", "<f4")])
SPHERE_DTYPE = np.dtype([("pos", "<f4", 3), ("radius", "<f4"), ("material", MATERIAL_DTYPE)])
LIGHT_DTYPE = np.dtype([("pos", "<f4", 3), ("col", "<f4", 3)])
assert VEC_DTYPE.itemsize == 12 and MATERIAL_DTYPE.itemsize == 32
assert SPHERE_DTYPE.itemsize == 48 and LIGHT_DTYPE.itemsize == 24

RTG_OK = 0
ERRORS = {-1: "invalid argument", -2: "HIP error", -3: "out of memory",
          -4: "no such device", -5: "I/O error"}

# Every symbol include/rtg.h declares (checked by tests/test_host.py).
EXPORTED = [
    "rtg_last_error", "rtg_abi_version", "rtg_device_count", "rtg_device_info",
    "rtg_render", "rtg_context_create", "rtg_context_destroy", "rtg_context_set_scene",
    "rtg_shard_rows", "rtg_shard_global_row", "rtg_render_device", "rtg_render_rows_device",
    "rtg_render_rows", "rtg_set_launch_opts", "rtg_diag_read", "rtg_diag_timeline", "rtg_diag_counts",
    "rtg_diag_group_list",
    "rtg_context_scene_stats",
    "rtg_max_colour", "rtg_max_colour_device", "rtg_ppm_bytes", "rtg_ppm_bytes_device",
    "rtg_save_ppm", "rtg_make_material", "rtg_scene_generate", "rtg_assemble_shards_device",
    "rtg_render_multi", "rtg_scene_load", "rtg_scene_save", "rtg_context_set_semantics",
    "rtg_multi_create", "rtg_multi_set_scene", "rtg_multi_render", "rtg_multi_destroy",
    "rtg_multi_set_gather", "rtg_place_shard_device",
]


# Counter slots of the traversal (rtg_trace.h kCnt* then the kU* executed-work
# units), the order of rtg_diag_counts / hostsim_counts.
UNIT_NAMES = [
    "samples", "primQ", "primSel", "primCand", "enterQ", "enterOK", "fullQ", "fullCand",
    "shadowQ", "shadowSel", "shadowCand", "containMasked", "containSel", "containFull",
    "refraction", "reflPush", "bvhNodeTests", "bvhSphereTests", "coneQ", "coneSel",
    "bvhShadowQ", "bvhShadowNodeTests", "bvhShadowSphereTests",
    "U.query", "U.primIter", "U.primExact", "U.selIter", "U.selExact", "U.shdIter",
    "U.shdExact", "U.enterHead", "U.enterIter", "U.enterExact", "U.fullGroup", "U.fullExact",
    "U.bvhNode", "U.bvhSlot", "U.bvhExact", "U.contIter", "U.cont4", "U.contBvhNode", "U.cone",
    "U.maskIter", "U.node", "U.shade", "U.light", "U.shadow", "U.lit", "U.refr", "U.refrLeaf",
    "U.push", "U.descend", "U.unwind", "U.sample", "U.bvhPass",
    "U.capIter", "U.ovIter", "D.shdSame", "D.enterAll", "D.enterSame", "D.contSame",
    "U.lightDir", "D.insig", "D.insigAll", "U.wave",
]


class RtgError(RuntimeError):
    pass


_lib = None


def lib() -> ctypes.CDLL:
    """Load librtg.so (built in-tree by `make -C raytracer-gamma_amd`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RtgError(f"librtg.so not built at {LIB_PATH}; run __graft_entry__.build()")
        L = ctypes.CDLL(LIB_PATH)
        vp, u, i, f, sz = ctypes.c_void_p, ctypes.c_uint, ctypes.c_int, ctypes.c_float, ctypes.c_size_t
        L.rtg_last_error.restype = ctypes.c_char_p
        L.rtg_abi_version.restype = i
        L.rtg_device_count.argtypes = [ctypes.POINTER(i)]
        L.rtg_device_info.argtypes = [i, ctypes.c_char_p, sz]
        L.rtg_render.argtypes = [i, vp, u, vp, u, u, u, f, f, i, vp]
        L.rtg_context_create.argtypes = [i, ctypes.POINTER(vp)]
        L.rtg_context_destroy.argtypes = [vp]
        L.rtg_context_set_scene.argtypes = [vp, vp, u, vp, u]
        L.rtg_shard_rows.argtypes = [u, u, u, u, ctypes.POINTER(u)]
        L.rtg_shard_global_row.argtypes = [u, u, u, u]
        L.rtg_shard_global_row.restype = u
        L.rtg_render_device.argtypes = [vp, u, u, f, f, i, u, u, u, vp, vp]
        L.rtg_render_rows_device.argtypes = [vp, u, u, f, f, i, vp, u, vp, vp]
        L.rtg_render_rows.argtypes = [i, vp, u, vp, u, u, u, f, f, i, vp, u, vp]
        L.rtg_set_launch_opts.argtypes = [vp, vp]
        L.rtg_context_set_semantics.argtypes = [vp, i]
        L.rtg_diag_read.argtypes = [vp, vp, i]
        L.rtg_diag_timeline.argtypes = [vp, vp, sz, vp]
        if hasattr(L, "rtg_diag_group_list"):  # (A/B libraries of older revisions lack it)
            L.rtg_diag_group_list.argtypes = [vp, vp, vp, vp, vp, sz, vp]
        # round-3 entry points; an RTG_LIB build from before them (same-box A/B
        # of older kernels, tools/ab_bench.sh) loads without them
        for name, at in (("rtg_diag_counts", [vp, vp, i, i]),
                         ("rtg_context_scene_stats", [vp, vp]),
                         ("rtg_multi_set_gather", [vp, i]),
                         ("rtg_place_shard_device", [vp, vp, u, u, u, u, u, vp, vp])):
            try:
                getattr(L, name).argtypes = at
            except AttributeError:
                if not os.environ.get("RTG_LIB"):
                    raise
        L.rtg_max_colour.argtypes = [vp, sz]
        L.rtg_max_colour.restype = f
        L.rtg_max_colour_device.argtypes = [vp, vp, sz, vp, vp]
        L.rtg_ppm_bytes.argtypes = [vp, sz, f, vp]
        L.rtg_ppm_bytes.restype = None
        L.rtg_ppm_bytes_device.argtypes = [vp, vp, sz, vp, vp, vp]
        L.rtg_assemble_shards_device.argtypes = [vp, vp, u, u, u, u, u, vp, vp]
        L.rtg_render_multi.argtypes = [vp, i, vp, u, vp, u, u, u, f, f, i, u, vp, vp]
        L.rtg_multi_create.argtypes = [vp, i, ctypes.POINTER(vp)]
        L.rtg_multi_set_scene.argtypes = [vp, vp, u, vp, u]
        L.rtg_multi_render.argtypes = [vp, u, u, f, f, i, u, vp, vp]
        L.rtg_multi_destroy.argtypes = [vp]

        pu = ctypes.POINTER(u)
        L.rtg_scene_load.argtypes = [ctypes.c_char_p, vp, u, pu, vp, u, pu]
        L.rtg_scene_save.argtypes = [ctypes.c_char_p, vp, u, vp, u]
        L.rtg_save_ppm.argtypes = [vp, ctypes.c_char_p, i, i, f]
        L.rtg_make_material.argtypes = [f, f, vp, vp, f, vp]
        L.rtg_make_material.restype = None
        L.rtg_scene_generate.argtypes = [ctypes.c_ulonglong, u, u, vp, vp]
        _lib = L
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != RTG_OK:
        msg = lib().rtg_last_error().decode(errors="replace")
        raise RtgError(f"{what}: {ERRORS.get(rc, rc)}: {msg}")


def _ptr(a: np.ndarray):
    return ctypes.c_void_p(a.ctypes.data) if a is not None and a.size else None


# ---------------------------------------------------------------- scene helpers
def make_material(opacity, gloss_factor, matte, gloss, refractive_index):
    """setMatOpacity + setMatteGlossBalance + setMatRefractivityIndex (raytracer.h:53-74)."""
    out = np.zeros(1, MATERIAL_DTYPE)
    m = np.asarray(matte, np.float32)
    g = np.asarray(gloss, np.float32)
    lib().rtg_make_material(float(opacity), float(gloss_factor), _ptr(m), _ptr(g),
                            float(refractive_index), _ptr(out))
    return out[0]


def generate_scene(n_spheres: int, n_lights: int, seed: int = 42):
    """main.cpp:104-168 scene, extended by the seeded generator of SURVEY.md §8d."""
    sph = np.zeros(n_spheres, SPHERE_DTYPE)
    lgt = np.zeros(n_lights, LIGHT_DTYPE)
    _check(lib().rtg_scene_generate(seed, n_spheres, n_lights, _ptr(sph), _ptr(lgt)),
           "rtg_scene_generate")
    return sph, lgt


def load_scene_file(path: str):
    """Spheres and lights of a scene file (rtg_scene_load; format in include/rtg.h)."""
    n, m = ctypes.c_uint(0), ctypes.c_uint(0)
    _check(lib().rtg_scene_load(path.encode(), None, 0, ctypes.byref(n), None, 0,
                                ctypes.byref(m)), "rtg_scene_load")
    sph = np.zeros(n.value, SPHERE_DTYPE)
    lgt = np.zeros(m.value, LIGHT_DTYPE)
    _check(lib().rtg_scene_load(path.encode(), _ptr(sph), n.value, ctypes.byref(n), _ptr(lgt),
                                m.value, ctypes.byref(m)), "rtg_scene_load")
    return sph, lgt


def save_scene_file(path: str, spheres, lights) -> None:
    spheres = np.ascontiguousarray(spheres, SPHERE_DTYPE)
    lights = np.ascontiguousarray(lights, LIGHT_DTYPE)
    _check(lib().rtg_scene_save(path.encode(), _ptr(spheres), len(spheres), _ptr(lights),
                                len(lights)), "rtg_scene_save")


def reference_scene():
    """The scene hard-coded in main.cpp:104-168 (3 spheres, 2 lights)."""
    return generate_scene(3, 2)


# ---------------------------------------------------------------- output helpers
def max_colour_value(fb: np.ndarray) -> float:
    """maxColourValuePixelBuffer, algebra.h:68-91."""
    fb = np.ascontiguousarray(fb, np.float32)
    return float(lib().rtg_max_colour(_ptr(fb), fb.size // 3))


def ppm_bytes(fb: np.ndarray, max_colour: float) -> np.ndarray:
    fb = np.ascontiguousarray(fb, np.float32)
    out = np.empty(fb.size, np.uint8)
    lib().rtg_ppm_bytes(_ptr(fb), fb.size // 3, float(max_colour), _ptr(out))
    return out


def ppm_file_bytes(fb: np.ndarray, max_colour: float | None = None) -> bytes:
    """Exact bytes savePPM (main.cpp:43-91) writes for an (H, W, 3) framebuffer."""
    h, w = fb.shape[0], fb.shape[1]
    mx = max_colour_value(fb) if max_colour is None else max_colour
    return b"P6\n%d %d\n255\n" % (w, h) + ppm_bytes(fb, mx).tobytes()


def save_ppm(fb: np.ndarray, filename: str, max_colour: float | None = None) -> None:
    fb = np.ascontiguousarray(fb, np.float32)
    mx = max_colour_value(fb) if max_colour is None else max_colour
    _check(lib().rtg_save_ppm(_ptr(fb), filename.encode(), fb.shape[1], fb.shape[0], mx),
           "rtg_save_ppm")


def shard_rows(height: int, row_block: int, shard: int, n_shards: int) -> int:
    r = ctypes.c_uint(0)
    _check(lib().rtg_shard_rows(height, row_block, shard, n_shards, ctypes.byref(r)),
           "rtg_shard_rows")
    return r.value


def shard_row_indices(height: int, row_block: int, shard: int, n_shards: int) -> np.ndarray:
    n = shard_rows(height, row_block, shard, n_shards)
    f = lib().rtg_shard_global_row
    return np.array([f(k, row_block, shard, n_shards) for k in range(n)], np.int64)


# ---------------------------------------------------------------- device
def device_count() -> int:
    c = ctypes.c_int(0)
    _check(lib().rtg_device_count(ctypes.byref(c)), "rtg_device_count")
    return c.value


def device_info(device: int = 0) -> str:
    buf = ctypes.create_string_buffer(256)
    _check(lib().rtg_device_info(device, buf, 256), "rtg_device_info")
    return buf.value.decode()


def render(spheres, lights, width: int, height: int, zoom: float = -4.0,
           alias_factor: float = 3.0, stack_size: int = 6, device: int = 0) -> np.ndarray:
    """One-shot drop-in for the reference's GPU launch (main.cpp:277-468):
    returns the (H, W, 3) float32 framebuffer of the reference CPU path."""
    spheres = np.ascontiguousarray(spheres, SPHERE_DTYPE)
    lights = np.ascontiguousarray(lights, LIGHT_DTYPE)
    out = np.empty((height, width, 3), np.float32)
    _check(lib().rtg_render(device, _ptr(spheres), len(spheres), _ptr(lights), len(lights),
                            width, height, float(zoom), float(alias_factor), stack_size,
                            _ptr(out)), "rtg_render")
    return out


def render_multi(spheres, lights, width: int, height: int, devices=(0,), zoom: float = -4.0,
                 alias_factor: float = 3.0, stack_size: int = 6, row_block: int = 16):
    """Multi-GPU one-shot in ONE process (rtg_render_multi): row-cyclic shards on
    `devices`, one RCCL gather to devices[0].  Returns (frame, timings_ms) with
    timings = [slowest render, gather + assemble, wall]."""
    spheres = np.ascontiguousarray(spheres, SPHERE_DTYPE)
    lights = np.ascontiguousarray(lights, LIGHT_DTYPE)
    devs = np.ascontiguousarray(devices, np.int32)
    out = np.empty((height, width, 3), np.float32)
    tm = np.zeros(3, np.float32)
    _check(lib().rtg_render_multi(_ptr(devs), len(devs), _ptr(spheres), len(spheres),
                                  _ptr(lights), len(lights), width, height, float(zoom),
                                  float(alias_factor), stack_size, row_block, _ptr(out),
                                  _ptr(tm)), "rtg_render_multi")
    return out, [float(v) for v in tm]


class MultiContext:
    """Persistent multi-device handle (rtg_multi_*): RCCL communicator, contexts,
    streams and buffers kept across frames."""

    def __init__(self, devices=(0,)):
        self._h = ctypes.c_void_p()
        self._devs = np.ascontiguousarray(devices, np.int32)
        _check(lib().rtg_multi_create(_ptr(self._devs), len(self._devs), ctypes.byref(self._h)),
               "rtg_multi_create")

    def set_scene(self, spheres, lights):
        self._sph = np.ascontiguousarray(spheres, SPHERE_DTYPE)
        self._lgt = np.ascontiguousarray(lights, LIGHT_DTYPE)
        _check(lib().rtg_multi_set_scene(self._h, _ptr(self._sph), len(self._sph),
                                         _ptr(self._lgt), len(self._lgt)), "rtg_multi_set_scene")

    GATHER_RCCL, GATHER_PEER_COPY = 0, 1  # RTG_GATHER_*

    def set_gather(self, mode: int):
        """RCCL gather + assemble (default) or the peer-copy ablation."""
        _check(lib().rtg_multi_set_gather(self._h, int(mode)), "rtg_multi_set_gather")

    def render(self, width, height, zoom=-4.0, alias_factor=3.0, stack_size=6, row_block=16):
        out = np.empty((height, width, 3), np.float32)
        tm = np.zeros(3, np.float32)
        _check(lib().rtg_multi_render(self._h, width, height, float(zoom), float(alias_factor),
                                      stack_size, row_block, _ptr(out), _ptr(tm)),
               "rtg_multi_render")
        return out, [float(v) for v in tm]

    def close(self):
        if self._h:
            lib().rtg_multi_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def render_rows(spheres, lights, width: int, height: int, rows, zoom: float = -4.0,
                alias_factor: float = 3.0, stack_size: int = 6, device: int = 0) -> np.ndarray:
    """Render only the listed global rows; returns (len(rows), W, 3)."""
    spheres = np.ascontiguousarray(spheres, SPHERE_DTYPE)
    lights = np.ascontiguousarray(lights, LIGHT_DTYPE)
    rows = np.ascontiguousarray(rows, np.uint32)
    out = np.empty((len(rows), width, 3), np.float32)
    _check(lib().rtg_render_rows(device, _ptr(spheres), len(spheres), _ptr(lights),
                                 len(lights), width, height, float(zoom), float(alias_factor),
                                 stack_size, _ptr(rows), len(rows), _ptr(out)),
           "rtg_render_rows")
    return out


class Context:
    """Persistent device context: scene resident in HBM, renders into caller
    device memory (e.g. a torch tensor's data_ptr()) on a caller stream."""

    def __init__(self, device: int = 0):
        self._h = ctypes.c_void_p()
        _check(lib().rtg_context_create(device, ctypes.byref(self._h)), "rtg_context_create")
        self.device = device

    def close(self):
        if self._h:
            lib().rtg_context_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def set_scene(self, spheres, lights):
        self._sph = np.ascontiguousarray(spheres, SPHERE_DTYPE)
        self._lgt = np.ascontiguousarray(lights, LIGHT_DTYPE)
        _check(lib().rtg_context_set_scene(self._h, _ptr(self._sph), len(self._sph),
                                           _ptr(self._lgt), len(self._lgt)),
               "rtg_context_set_scene")

    def scene_stats(self):
        """{prep_ms, upload_ms, device_bytes, bvh_nodes} of the last set_scene."""
        if not hasattr(lib(), "rtg_context_scene_stats"):  # an older RTG_LIB build
            return {"prep_ms": 0.0, "upload_ms": 0.0, "device_bytes": 0, "bvh_nodes": 0}
        out = (ctypes.c_double * 4)()
        _check(lib().rtg_context_scene_stats(self._h, ctypes.cast(out, ctypes.c_void_p)),
               "rtg_context_scene_stats")
        return {"prep_ms": out[0], "upload_ms": out[1], "device_bytes": int(out[2]),
                "bvh_nodes": int(out[3])}

    LAUNCH_TIMELINE = 1  # RTG_LAUNCH_TIMELINE
    LAUNCH_NO_ORDER_FEEDBACK = 2  # RTG_LAUNCH_NO_ORDER_FEEDBACK
    SEMANTICS_CPU, SEMANTICS_OPENCL = 0, 1  # RTG_SEMANTICS_*

    def set_semantics(self, semantics: int):
        """CPU path (default, bit-exact) or the reference OpenCL kernel's semantics."""
        _check(lib().rtg_context_set_semantics(self._h, int(semantics)),
               "rtg_context_set_semantics")

    def set_variant(self, variant: int, flags: int = 0):
        opts = (ctypes.c_int * 8)(variant, flags, 0, 0, 0, 0, 0, 0)
        _check(lib().rtg_set_launch_opts(self._h, ctypes.cast(opts, ctypes.c_void_p)),
               "rtg_set_launch_opts")

    def diag_read(self, reset: bool = True):
        out = (ctypes.c_ulonglong * 8)()
        _check(lib().rtg_diag_read(self._h, ctypes.cast(out, ctypes.c_void_p), int(reset)),
               "rtg_diag_read")
        return [int(v) for v in out]

    def diag_counts(self, reset: bool = True):
        """Executed-work unit counters of the counting build (variant 120):
        (wave-level, lane-level) arrays indexed by UNIT_NAMES."""
        n = lib().rtg_diag_counts(self._h, None, 0, 0)
        if n < 0:
            _check(n, "rtg_diag_counts")
        out = (ctypes.c_ulonglong * n)()
        rc = lib().rtg_diag_counts(self._h, ctypes.cast(out, ctypes.c_void_p), n, int(reset))
        if rc < 0:
            _check(rc, "rtg_diag_counts")
        v = np.array(out[:], np.int64)
        return v[:n // 2], v[n // 2:]

    def diag_timeline(self, cap: int = 1 << 20) -> np.ndarray:
        """Per-wave records {start, end, HW_ID, XCC_ID} of the last timeline-variant launch."""
        out = np.zeros((cap, 4), np.uint32)
        cnt = ctypes.c_size_t(0)
        _check(lib().rtg_diag_timeline(self._h, ctypes.c_void_p(out.ctypes.data), cap,
                                       ctypes.byref(cnt)), "rtg_diag_timeline")
        return out[:min(cap, cnt.value)]

    def diag_group_list(self, cap: int = 1 << 26):
        """The last compacted launch: {cost[groups], list[listed], sel[listed],
        runs[4]}, list and sel in the trace kernel's order (rtg_diag_group_list;
        costs in 100 MHz ticks)."""
        n = ctypes.c_size_t(0)
        _check(lib().rtg_diag_group_list(self._h, None, None, None, None, 0, ctypes.byref(n)),
               "rtg_diag_group_list")
        g = min(cap, n.value)
        cost = np.zeros(g, np.uint32)
        lst = np.zeros(g, np.uint32)
        sel = np.zeros(g, np.uint64)
        runs = np.zeros(4, np.uint32)
        _check(lib().rtg_diag_group_list(self._h, ctypes.c_void_p(cost.ctypes.data),
                                         ctypes.c_void_p(lst.ctypes.data),
                                         ctypes.c_void_p(sel.ctypes.data),
                                         ctypes.c_void_p(runs.ctypes.data), g, ctypes.byref(n)),
               "rtg_diag_group_list")
        k = int(runs.sum())
        return {"cost": cost, "list": lst[:k], "sel": sel[:k], "runs": runs}

    def render_device(self, width, height, dst_ptr: int, zoom=-4.0, alias_factor=3.0,
                      stack_size=6, row_block=16, shard=0, n_shards=1, stream: int = 0):
        _check(lib().rtg_render_device(self._h, width, height, float(zoom),
                                       float(alias_factor), stack_size, row_block, shard,
                                       n_shards, ctypes.c_void_p(dst_ptr),
                                       ctypes.c_void_p(stream) if stream else None),
               "rtg_render_device")

    def render_rows_device(self, width, height, rows_ptr: int, n_rows: int, dst_ptr: int,
                           zoom=-4.0, alias_factor=3.0, stack_size=6, stream: int = 0):
        """Render the global rows listed at rows_ptr (device uint32[n_rows])."""
        _check(lib().rtg_render_rows_device(self._h, width, height, float(zoom),
                                            float(alias_factor), stack_size,
                                            ctypes.c_void_p(rows_ptr), n_rows,
                                            ctypes.c_void_p(dst_ptr),
                                            ctypes.c_void_p(stream) if stream else None),
               "rtg_render_rows_device")

    def max_colour_device(self, src_ptr: int, n_pixels: int, dst_ptr: int, stream: int = 0):
        _check(lib().rtg_max_colour_device(self._h, ctypes.c_void_p(src_ptr), n_pixels,
                                           ctypes.c_void_p(dst_ptr),
                                           ctypes.c_void_p(stream) if stream else None),
               "rtg_max_colour_device")

    def assemble_shards_device(self, gathered_ptr: int, n_shards: int, padded_rows: int,
                               width: int, height: int, row_block: int, frame_ptr: int,
                               stream: int = 0):
        """Row order back from gathered row-cyclic shards (rtg_assemble_shards_device)."""
        _check(lib().rtg_assemble_shards_device(self._h, ctypes.c_void_p(gathered_ptr), n_shards,
                                                padded_rows, width, height, row_block,
                                                ctypes.c_void_p(frame_ptr),
                                                ctypes.c_void_p(stream) if stream else None),
               "rtg_assemble_shards_device")

    def place_shard_device(self, shard_ptr: int, shard: int, n_shards: int, width: int,
                           height: int, row_block: int, frame_ptr: int, stream: int = 0):
        """Copy one shard's packed rows into their rows of a frame (rtg_place_shard_device)."""
        _check(lib().rtg_place_shard_device(self._h, ctypes.c_void_p(shard_ptr), shard, n_shards,
                                            width, height, row_block, ctypes.c_void_p(frame_ptr),
                                            ctypes.c_void_p(stream) if stream else None),
               "rtg_place_shard_device")

    def ppm_bytes_device(self, src_ptr: int, n_pixels: int, max_ptr: int, dst_ptr: int,
                         stream: int = 0):
        _check(lib().rtg_ppm_bytes_device(self._h, ctypes.c_void_p(src_ptr), n_pixels,
                                          ctypes.c_void_p(max_ptr), ctypes.c_void_p(dst_ptr),
                                          ctypes.c_void_p(stream) if stream else None),
               "rtg_ppm_bytes_device")


def canonical_bits(fb: np.ndarray) -> np.ndarray:
    """uint32 view with every NaN mapped to the x86 default NaN 0xFFC00000."""
    b = np.ascontiguousarray(fb, np.float32).view(np.uint32).copy()
    b[np.isnan(np.ascontiguousarray(fb, np.float32))] = 0xFFC00000
    return b
