"""CPU tests of the product's host runtime behind the C-ABI (no GPU needed):
the library loads and exports every function include/srr_capi.h declares,
the host pieces that feed the kernels (teapot tessellation, the
reference-topology BVH builder, Sobol points) match the REFERENCE's goldens
bit for bit, and the renderer refuses to run without a HIP device (no CPU
fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_bind as ob
from srr import capi, scenes

ROOT = ob.ROOT
HEADER = os.path.join(ROOT, "include", "srr_capi.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(srr_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    L = capi.lib()
    names = declared_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert b"srr" in L.srr_version()


def test_teapot_tessellation_matches_reference():
    L = capi.lib()
    L.srr_teapot_vertices.argtypes = [ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
    n = L.srr_teapot_vertices(60.0, 10, None)
    out = np.zeros((n, 9), np.float32)
    assert L.srr_teapot_vertices(60.0, 10, out.ctypes.data) == 6400
    g = np.fromfile(os.path.join(ob.GOLDEN, "teapot_s60_d10.f32"), np.float32).reshape(-1, 12)[:, :9]
    np.testing.assert_array_equal(out.view(np.uint32), g.view(np.uint32))


def _bvh_text(scene_text, text_id):
    L = capi.lib()
    L.srr_scene_text_handle.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.srr_bvh_topology.restype = ctypes.c_int64
    L.srr_bvh_topology.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int64]
    sc = capi.Scene(scene_text)
    h = L.srr_scene_text_handle(sc.h, text_id)
    assert h >= 0
    n = L.srr_bvh_topology(sc.h, h, None, 0)
    buf = ctypes.create_string_buffer(int(n))
    L.srr_bvh_topology(sc.h, h, buf, n)
    return buf.value.decode()


def test_bvh_topology_matches_reference():
    """bvh_node's random-axis median split with glibc qsort order."""
    text = open(os.path.join(ob.GOLDEN, "s2.scene")).read()
    got = _bvh_text(text, 11).splitlines()
    want = open(os.path.join(ob.GOLDEN, "bvh_s2_teapot.txt")).read().splitlines()
    assert len(got) == len(want)
    assert got[1:] == want[1:]
    gb = [float(x) for x in got[0].split()[1:]]
    wb = [float(x) for x in want[0].split()[1:]]
    np.testing.assert_allclose(gb, wb, rtol=1e-5)


def test_sobol_matches_reference():
    for n in (64, 1024, 4096):
        g = np.fromfile(os.path.join(ob.GOLDEN, f"sobol_{n}.f64"), np.float64).reshape(n, 2)
        np.testing.assert_array_equal(capi.sobol_points(n), g)


@pytest.mark.parametrize("name", ["s1", "s2", "s3", "s4_small", "s5_small"])
def test_scene_text_parses(name):
    capi.Scene(open(os.path.join(ob.GOLDEN, f"{name}.scene")).read())


def test_bad_scene_is_an_error_not_a_crash():
    with pytest.raises(capi.SrrError):
        capi.Scene("srr_scene 1\nobj 0 sphere 0 0 0 1 7\n")  # undefined material 7
    with pytest.raises(capi.SrrError):
        capi.Scene("not a scene")


def test_shard_pixels_partition_the_image():
    nx, ny = 100, 70
    seen = np.zeros(nx * ny, np.int32)
    for k in range(3):
        px = capi.shard_pixels(capi.make_params(nx, ny, 1, shard=(k, 3), tile=32))
        assert np.all(np.diff(px) > 0)
        seen[px] += 1
    assert np.all(seen == 1)


def test_renderer_without_gpu_fails_loudly():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    sc, _ = scenes.s1_cornell()
    with pytest.raises(capi.SrrError, match="HIP device"):
        capi.Renderer(sc.text())
