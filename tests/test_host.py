"""CPU tests of librtg.so's host side: ABI surface, scene construction, PPM
writer, colour max, row sharding and error behaviour.  No GPU calls."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, P, PKG, ROOT, load_scene, md5


def _declared_functions():
    src = open(os.path.join(ROOT, "include", "rtg.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rtg_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol(rtg):
    declared = _declared_functions()
    assert len(declared) >= 20
    lib = rtg.lib()
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    assert sorted(rtg.EXPORTED) == declared
    assert lib.rtg_abi_version() == 1


def test_struct_layouts_match_reference(rtg):
    # vec.h / material.h / sphere.h / raytracer.h:20-25 (also static_asserted in C++)
    assert rtg.SPHERE_DTYPE.fields["radius"][1] == 12
    assert rtg.SPHERE_DTYPE.fields["material"][1] == 16
    assert rtg.MATERIAL_DTYPE.fields["opacity"][1] == 24
    assert rtg.MATERIAL_DTYPE.fields["refractiveIndex"][1] == 28
    assert rtg.LIGHT_DTYPE.fields["col"][1] == 12


@pytest.mark.parametrize("name", ["ref800", "c1", "c2", "c3", "c4", "c5"])
def test_scene_generator_matches_golden(rtg, golden, name):
    c = golden["configs"][name]
    sph, lg = rtg.generate_scene(c["spheres"], c["lights"], 42)
    gs, gl = load_scene(name, c["spheres"], c["lights"])
    assert sph.tobytes() == gs.tobytes()
    assert lg.tobytes() == gl.tobytes()
    assert md5(sph.tobytes() + lg.tobytes()) == c["scene_md5"]


def test_main_cpp_materials(rtg):
    """main.cpp:126-145 via setMatteGlossBalance's double-precision factor."""
    sph, _ = rtg.reference_scene()
    m0 = sph[0]["material"]
    k = np.float32(1.0 - np.float64(np.float32(0.2)))
    assert m0["matteColour"][0] == k * np.float32(0.4)
    assert m0["glossColour"][1] == np.float32(0.2) * np.float32(1.0)
    assert m0["opacity"] == np.float32(0.8) and m0["refractiveIndex"] == np.float32(1.55)
    assert list(sph["radius"]) == [5.0, 2.0, 3.0]


def test_scene_generator_seeds_differ(rtg):
    a, _ = rtg.generate_scene(16, 3, 42)
    b, _ = rtg.generate_scene(16, 3, 43)
    assert a[:3].tobytes() == b[:3].tobytes()  # fixed main.cpp spheres
    assert a[3:].tobytes() != b[3:].tobytes()


def _special_floats(rng, n):
    v = rng.standard_normal(n).astype(np.float32) * np.float32(1e-4)
    specials = np.array([0.0, -0.0, np.nan, -np.nan, np.inf, -np.inf, 1.0, 2.0, 1e-38, 1e30,
                         -1e30, 0.99999994, 1.0000001, 7e-5, -7e-5, 3e38], np.float32)
    v[: len(specials)] = specials
    v[len(specials):len(specials) + 64] = rng.uniform(-2, 2, 64).astype(np.float32)
    return v


def test_ppm_bytes_match_oracle(rtg, oracle):
    rng = np.random.default_rng(3)
    fb = _special_floats(rng, 3 * 5000).reshape(-1, 3)
    for mx in [6.955025e-05, 1.0, 3.0535437e-05, 1e-30, 2.5]:
        a = rtg.ppm_bytes(fb, mx)
        b = oracle.ppm_bytes(fb, mx)
        assert (a == b).all()


def test_max_colour_matches_oracle(rtg, oracle):
    rng = np.random.default_rng(4)
    fb = _special_floats(rng, 3 * 777).reshape(-1, 3)
    fb[np.isinf(fb)] = 0  # keep a finite max for the second check below
    assert rtg.max_colour_value(fb) == oracle.max_colour(fb)
    assert rtg.max_colour_value(np.zeros((10, 3), np.float32)) == 1.0   # algebra.h:86-88
    assert rtg.max_colour_value(np.full((4, 3), np.nan, np.float32)) == 1.0
    assert rtg.max_colour_value(-np.ones((4, 3), np.float32)) == 1.0


@pytest.mark.parametrize("name", ["ref800", "c1"])
def test_save_ppm_matches_golden(rtg, oracle, golden, tmp_path, name):
    c = golden["configs"][name]
    sph, lg = load_scene(name, c["spheres"], c["lights"])
    fb = oracle.render(sph, lg, c["W"], c["H"], c["stack_size"])
    path = str(tmp_path / "out.ppm")
    rtg.save_ppm(fb, path)
    data = open(path, "rb").read()
    assert data[:15] == b"P6\n%d %d\n255\n" % (c["W"], c["H"])[:15]
    assert md5(data) == c["ppm_md5"]
    assert md5(rtg.ppm_file_bytes(fb)) == c["ppm_md5"]


def test_save_ppm_errors(rtg, tmp_path):
    with pytest.raises(rtg.RtgError):
        rtg.save_ppm(np.zeros((0, 4, 3), np.float32), str(tmp_path / "x.ppm"))
    with pytest.raises(rtg.RtgError):
        rtg.save_ppm(np.zeros((2, 2, 3), np.float32), str(tmp_path / "nodir" / "x.ppm"))


@pytest.mark.parametrize("H,B,G", [(2160, 16, 1), (2160, 16, 2), (2160, 16, 8), (2160, 8, 7),
                                   (600, 16, 3), (1, 16, 8), (17, 4, 5), (4320, 16, 8),
                                   (100, 1, 3), (33, 32, 2)])
def test_shard_rows_partition_frame(rtg, H, B, G):
    seen = []
    for g in range(G):
        rows = rtg.shard_row_indices(H, B, g, G)
        assert (np.diff(rows) > 0).all() if len(rows) > 1 else True
        for r in rows:
            assert (r // B) % G == g
        seen.extend(rows.tolist())
    assert sorted(seen) == list(range(H))


def test_shard_rows_invalid(rtg):
    with pytest.raises(rtg.RtgError):
        rtg.shard_rows(100, 0, 0, 1)
    with pytest.raises(rtg.RtgError):
        rtg.shard_rows(100, 16, 2, 2)


def test_render_entry_points_reject_bad_arguments_without_gpu(rtg):
    L = rtg.lib()
    # null context / scene: validated before any HIP call
    assert L.rtg_render_device(None, 8, 8, ctypes.c_float(-4), ctypes.c_float(3), 6, 16, 0, 1,
                               None, None) == -1
    assert L.rtg_render_rows_device(None, 8, 8, ctypes.c_float(-4), ctypes.c_float(3), 6,
                                    None, 3, None, None) == -1
    assert L.rtg_render(0, None, 0, None, 0, 4, 4, ctypes.c_float(-4), ctypes.c_float(3), 6,
                        None) == -1
    assert b"null" in L.rtg_last_error()
    assert L.rtg_context_set_scene(None, None, 0, None, 0) == -1


def test_host_driver_builds_and_prints_help():
    exe = os.path.join(PKG, "rtg_main")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", PKG, "rtg_main"], check=True)
    r = subprocess.run([exe, "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0
    assert "--width" in r.stdout and "--device" in r.stdout


# ------------------------------------------------------------------ scene files
def test_reference_scene_file_matches_main_cpp_scene(rtg):
    """scenes/reference.scene (built with the reference's material setters) is
    the scene of main.cpp:104-168 bit for bit, i.e. rtg_scene_generate(42, 3, 2)."""
    sph, lg = rtg.load_scene_file(os.path.join(ROOT, "scenes", "reference.scene"))
    want_s, want_l = rtg.reference_scene()
    assert sph.tobytes() == want_s.tobytes()
    assert lg.tobytes() == want_l.tobytes()


@pytest.mark.parametrize("n,m", [(0, 0), (3, 2), (16, 3), (1024, 4)])
def test_scene_file_round_trip(rtg, tmp_path, n, m):
    sph, lg = rtg.generate_scene(n, m, 7)
    rng = np.random.default_rng(n + m)
    if n:  # awkward floats too: subnormal, negative zero, huge, many digits
        sph["radius"][0] = np.float32(1.4e-45)
        sph["pos"][0, 0] = np.float32(-0.0)
        sph["material"]["opacity"][-1] = np.float32(3.4028235e38)
        sph["pos"][:, 1] = rng.standard_normal(n).astype(np.float32)
    path = str(tmp_path / "s.scene")
    rtg.save_scene_file(path, sph, lg)
    s2, l2 = rtg.load_scene_file(path)
    assert s2.tobytes() == sph.tobytes()
    assert l2.tobytes() == lg.tobytes()


def test_scene_file_errors_name_the_line(rtg, tmp_path):
    cases = {
        "sphere 1 2 3 4 nosuch\n": "unknown material",
        "material a 1 0 1 1 1 1 1 1\n": "expected: material",
        "light 1 2 3 4 5\n": "expected: light",
        "# ok\nsphere_raw 1 2 3\n": ":2:",
        "teapot 1 2 3\n": "unknown keyword",
        "light 1 2 3 4 5 x\n": "expected: light",
    }
    for text, msg in cases.items():
        p = tmp_path / "bad.scene"
        p.write_text(text)
        with pytest.raises(rtg.RtgError, match=re.escape(msg)):
            rtg.load_scene_file(str(p))
    with pytest.raises(rtg.RtgError, match="I/O error"):
        rtg.load_scene_file(str(tmp_path / "missing.scene"))


def test_scene_file_capacity_query(rtg, tmp_path):
    """Capacity 0 returns the totals; a short capacity loads a prefix."""
    sph, lg = rtg.generate_scene(5, 3, 1)
    path = str(tmp_path / "s.scene")
    rtg.save_scene_file(path, sph, lg)
    L = rtg.lib()
    n, m = ctypes.c_uint(0), ctypes.c_uint(0)
    assert L.rtg_scene_load(path.encode(), None, 0, ctypes.byref(n), None, 0, ctypes.byref(m)) == 0
    assert (n.value, m.value) == (5, 3)
    part = np.zeros(2, rtg.SPHERE_DTYPE)
    assert L.rtg_scene_load(path.encode(), ctypes.c_void_p(part.ctypes.data), 2, ctypes.byref(n),
                            None, 0, ctypes.byref(m)) == 0
    assert n.value == 5 and part.tobytes() == sph[:2].tobytes()


def test_host_driver_scene_options(tmp_path):
    """rtg_main --save-scene / --help (no GPU needed for these)."""
    exe = os.path.join(PKG, "rtg_main")
    if not os.path.exists(exe):
        pytest.skip("rtg_main not built")
    r = subprocess.run([exe, "--help"], capture_output=True, text=True)
    assert "--scene" in r.stdout and "--gpus" in r.stdout


def test_short_sequence_ranges_compose():
    """rcp_sqrt_rn (rtg_trace.h) takes rcp(sqrt(x)) with sqrt_fast's range check
    only, and make_query takes the reciprocal of 2|d|^2 with none: both rely on
    the rounded root / the Markstein denominator lying inside rcp_fast's range
    [2^-125, 2^125].  Check those bounds at the range ends in binary32."""
    f = np.float32
    lo, hi = f(2.0 ** -96), np.finfo(np.float32).max
    for x in (lo, np.nextafter(lo, f(1)), f(1), np.nextafter(hi, f(0)), hi):
        s = np.sqrt(f(x), dtype=np.float32)
        assert f(2.0 ** -125) <= s <= f(2.0 ** 125), (x, s)
    # the kFast quotient's denominator range (RayQ::fast) inside rcp_fast's
    assert 2.0 ** -125 <= 2.0 ** -60 and 2.0 ** 60 <= 2.0 ** 125
