"""Pins the CPU restatement oracle (oracle/restate.cpp) to the REFERENCE's own
outputs: every golden vector in tests/golden/ was produced by the reference
renderer's code (tests/golden/make_golden.py).  The restatement follows each
float/double promotion of the reference, so on this image's libm the
comparison is bit-exact."""
import json
import os

import numpy as np
import pytest

import oracle_bind as ob
import parity

META = json.load(open(os.path.join(ob.GOLDEN, "golden.json")))


@pytest.mark.parametrize("name", sorted(META["kats"]))
def test_kat_bitexact(name):
    rec = ob.read_kat(name)
    out = ob.replay_kat(name, rec)
    a = rec.view(np.uint32)
    b = out.view(np.uint32)
    bad = np.argwhere(a != b)
    assert bad.size == 0, f"{name}: {len(bad)} words differ, first at {bad[:5].tolist()}"


@pytest.mark.parametrize("name", sorted(META["renders"]))
def test_render_bitexact(name):
    m = META["renders"][name]
    text = open(os.path.join(ob.GOLDEN, f"{name}.scene")).read()
    r = ob.render(text, m["nx"], m["ny"], m["spp"], m["max_depth"])
    gp = np.fromfile(os.path.join(ob.GOLDEN, f"{name}.paths.f32"), np.float32).reshape(r["paths"].shape)
    gr = np.fromfile(os.path.join(ob.GOLDEN, f"{name}.rays.u8"), np.uint8).reshape(r["rays"].shape)
    gi = np.fromfile(os.path.join(ob.GOLDEN, f"{name}.img.f32"), np.float32).reshape(r["img"].shape)
    assert int(r["stats"][0]) == m["world_rays"]
    np.testing.assert_array_equal(r["rays"], gr)
    same = (r["paths"].view(np.uint32) == gp.view(np.uint32))
    assert same.all(), f"{(~same).sum()} path words differ"
    np.testing.assert_array_equal(r["img"].view(np.uint32), gi.view(np.uint32))


def test_sobol_matches_reference():
    for n in (64, 1024, 4096):
        g = np.fromfile(os.path.join(ob.GOLDEN, f"sobol_{n}.f64"), np.float64).reshape(n, 2)
        np.testing.assert_array_equal(ob.sobol(n), g)


def test_teapot_vertices_match_reference():
    g = np.fromfile(os.path.join(ob.GOLDEN, "teapot_s60_d10.f32"), np.float32).reshape(-1, 12)
    t = ob.teapot(60.0, 10)
    assert t.shape == g.shape == (6400, 12)
    np.testing.assert_array_equal(t.view(np.uint32), g.view(np.uint32))


def test_render_threads_deterministic():
    text = open(os.path.join(ob.GOLDEN, "s2.scene")).read()
    a = ob.render(text, 16, 16, 4, 50, threads=1)
    b = ob.render(text, 16, 16, 4, 50, threads=4)
    np.testing.assert_array_equal(a["paths"].view(np.uint32), b["paths"].view(np.uint32))


def test_restatement_matches_reference_tail_pixels():
    """The C2 frame's NaN-bound pixels (tests/golden/make_tail.py: a ray in the
    light's plane makes closest_so_far NaN before the teapot is tested): the
    restatement's paths are the reference's, bit for bit."""
    meta = json.load(open(os.path.join(ob.GOLDEN, "c2_tail.json")))
    text = open(os.path.join(ob.GOLDEN, meta["scene"])).read()
    pix = np.array(meta["pixels"], np.int32)
    n, spp = len(pix), meta["spp"]
    gp = np.fromfile(os.path.join(ob.GOLDEN, "c2_tail.paths.f32"), np.float32).reshape(n, spp, 3)
    gr = np.fromfile(os.path.join(ob.GOLDEN, "c2_tail.rays.u8"), np.uint8).reshape(n, spp)
    r = ob.render(text, meta["nx"], meta["ny"], spp, meta["max_depth"], pixels=pix, threads=8)
    pc = parity.compare_paths(r["paths"], gp)
    assert pc["bitexact"] == 1.0, pc
    assert (r["rays"] == gr).all()
    assert int(r["stats"][0]) == meta["world_rays"]
