"""The resampling loop's attempt cap (DESIGN §2 build definitions).

The reference's ``while (pdf_val == 0)`` (Raytracing_n.cpp:79-83) has no bound;
from a hit point coplanar with a triangle light it never ends (scenes.s7:
every light sample is rejected by ``triangle::hit``'s det < 1e-4 test and every
BSDF value is 0).  The product (kernels.hip kMixtureGuard) and the restatement
(oracle/restate.cpp kMixtureGuard) share one definition: stop after 100,000
attempts and keep the last one (pdf 0; the record's division gives inf/NaN,
which de_nan zeroes).  The reference itself cannot produce a golden here (it
hangs), so the restatement is the checker -- parity on these paths is pinned
to the restatement only.
"""
import json
import os

import numpy as np
import pytest

import oracle_bind as ob
import parity
from srr import capi, scenes

GUARD = 100000


def _oracle_s7():
    sc, c = scenes.s7_coplanar_light()
    text = sc.text()
    return text, c, ob.render(text, c["nx"], c["ny"], c["spp"], c["max_depth"], threads=8)


def test_oracle_caps_coplanar_light_loops():
    """The restatement stops each never-ending loop at the cap: the scene drives
    it (capped loops counted), and the capped paths carry the inf/NaN of the
    pdf-0 record while every other path stays finite-or-NaN as the reference's."""
    _, c, r = _oracle_s7()
    capped = int(r["stats"][4])
    assert capped > 50, r["stats"]
    nan_paths = int(np.isnan(r["paths"]).any(-1).sum())
    assert nan_paths > 0
    # the cap is per loop: the world rays stay those of the paths' bounces
    assert int(r["stats"][0]) == int(r["rays"].sum())


def test_guard_constant_shared():
    """One definition in the restatement and the product sources."""
    root = os.path.join(os.path.dirname(__file__), "..")
    src_o = open(os.path.join(root, "oracle", "restate.cpp")).read()
    src_k = open(os.path.join(root, "simple-raytracing-render_amd", "csrc", "kernels.hip")).read()
    assert f"constexpr int kMixtureGuard = {GUARD};" in src_o
    assert f"constexpr int kMixtureGuard = {GUARD};" in src_k
    assert "guard < kMixtureGuard" in src_k


@pytest.mark.gpu
@pytest.mark.parametrize("engine", ["paths", "wavefront", "paths_deep0"])
def test_gpu_capped_loops_match_restatement(engine, monkeypatch):
    """Every path of the coplanar-light scene bit-identical to the restatement,
    the same world rays, and (path engine) the same number of capped loops.
    paths_deep0: SRR_DEEP_TRIES=0 sends every pending loop straight to the
    all-64-lanes branch of coop_mixture."""
    text, c, r = _oracle_s7()
    if engine == "paths_deep0":
        monkeypatch.setenv("SRR_DEEP_TRIES", "0")
    flags = capi.FLAG_WAVEFRONT if engine == "wavefront" else 0
    out = capi.Renderer(text).render(c["nx"], c["ny"], c["spp"], c["max_depth"], keep_paths=True, flags=flags)
    pc = parity.compare_paths(out["paths"], r["paths"])
    print(engine, pc, "capped", out["stats"]["mixture_capped"], "oracle", int(r["stats"][4]))
    assert pc["bitexact"] >= parity.MIN_BITEXACT, pc
    assert (out["rays"] == r["rays"]).all()
    assert out["stats"]["world_rays"] == int(r["stats"][0])
    if engine != "wavefront":
        assert out["stats"]["mixture_capped"] == int(r["stats"][4])


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["s6_lights", "s2", "s4_d40"])
def test_gpu_deep_tries_zero_matches_reference(name, monkeypatch):
    """coop_mixture's all-lanes branch (normally taken only after 32 failed
    attempts) forced from the first round: the reference's goldens, bit for bit."""
    monkeypatch.setenv("SRR_DEEP_TRIES", "0")
    meta = json.load(open(os.path.join(ob.GOLDEN, "golden.json")))["renders"][name]
    n = meta["nx"] * meta["ny"]
    text = open(os.path.join(ob.GOLDEN, f"{name}.scene")).read()
    gp = np.fromfile(os.path.join(ob.GOLDEN, f"{name}.paths.f32"), np.float32).reshape(n, meta["spp"], 3)
    out = capi.Renderer(text).render(meta["nx"], meta["ny"], meta["spp"], meta["max_depth"], keep_paths=True)
    pc = parity.compare_paths(out["paths"], gp)
    assert pc["bitexact"] >= parity.MIN_BITEXACT, pc
    assert out["stats"]["world_rays"] == meta["world_rays"]
    assert out["stats"]["mixture_capped"] == 0
