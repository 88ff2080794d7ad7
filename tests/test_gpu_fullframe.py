"""GPU parity on the FULL headline frame: C2 (Cornell box + 6,400-tri teapot,
512x512x1024, maxDepth 50) rendered by the HIP path through the C-ABI, every
one of its 268 M paths checked bit for bit against the reference's own render
of the same frame via per-pixel digests (tests/golden/c2_full.npz, made by
oracle/_ref/ref_harness; tests/fullframe.py).  Exact equality: world-ray sums,
per-path radiance bits (NaN payloads aside) and the mean image.

On a mismatch, with SRR_DIAG_DIR set, the failing pixels' per-path outputs are
saved there for bisection against the CPU restatement (tools/diag_fullframe.py)."""
import json
import os

import numpy as np
import pytest

import fullframe
import parity
from srr import capi

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

pytestmark = pytest.mark.gpu


def _save_diag(name, bad, out):
    d = os.environ.get("SRR_DIAG_DIR")
    if not d or bad.size == 0:
        return
    os.makedirs(d, exist_ok=True)
    bad = bad[:4096]
    np.savez_compressed(os.path.join(d, f"{name}_diff.npz"), pixels=bad, paths=out["paths"][bad],
                        rays=out["rays"][bad], mean=out["mean"][bad])


@pytest.mark.parametrize("mode", ["default", "quad", "deep0"])
def test_c2_full_frame_is_the_reference_frame(mode, monkeypatch):
    """quad forces the quad-cooperative mesh traversal (kernels.hip
    mesh_hit4_quad) onto the L2-resident teapot, which by default runs per lane;
    deep0 (SRR_DEEP_TRIES=0) sends every resampling loop to coop_mixture's
    all-64-lanes branch from its first cooperative round."""
    monkeypatch.setenv("SRR_QUAD", "1" if mode == "quad" else "0")
    if mode == "deep0":
        monkeypatch.setenv("SRR_DEEP_TRIES", "0")
    name = "c2_full"
    m = fullframe.meta(name)
    want = fullframe.load(name)
    r = capi.Renderer(fullframe.scene_text(name))
    out = r.render(m["nx"], m["ny"], m["spp"], m["max_depth"], keep_paths=True)
    got = fullframe.digest(out["paths"], out["rays"])
    got["mean"] = out["mean"]
    res = fullframe.compare(got, want)
    res["stats_world_rays"] = out["stats"]["world_rays"]
    print(name, res)
    bad = np.flatnonzero((got["hash"] != want["hash"]) | (got["rays"] != want["rays"]))
    _save_diag(name, bad, out)
    assert out["stats"]["world_rays"] == m["world_rays"], res
    assert res["ray_mismatch_pixels"] == 0 and res["hash_mismatch_pixels"] == 0, res
    assert res["mean_mismatch_pixels"] == 0, res
    # the tail pixels (NaN-bound world hits, tests/golden/make_tail.py): every
    # path's radiance bits and world rays against the reference's own paths
    tail = json.load(open(os.path.join(GOLDEN, "c2_tail.json")))
    tp = np.array(tail["pixels"])
    gp = np.fromfile(os.path.join(GOLDEN, "c2_tail.paths.f32"), np.float32).reshape(len(tp), tail["spp"], 3)
    gr = np.fromfile(os.path.join(GOLDEN, "c2_tail.rays.u8"), np.uint8).reshape(len(tp), tail["spp"])
    pc = parity.compare_paths(out["paths"][tp], gp)
    assert pc["bitexact"] == 1.0, pc
    assert (out["rays"][tp] == gr).all()


@pytest.mark.parametrize("name", ["c4_full", "c5_full", "c4r_full"])
def test_1080p_full_frame_is_the_reference_frame(name):
    """The 1920x1080 configs' WHOLE frames at 16 spp (33 M paths each): C4 and
    C5 (the BASELINE stand-ins with the 102,400-triangle mesh; C5 adds the fog)
    and C4_real (the reference's own soldier_scene, Raytracing_n.cpp:585-657,
    from its committed fixture), every path's radiance bits and world rays
    against the reference's own render (grouped digests, tests/fullframe.fold)."""
    m = fullframe.meta(name)
    want = fullframe.load(name)
    r = capi.Renderer(fullframe.scene_text(name))
    out = r.render(m["nx"], m["ny"], m["spp"], m["max_depth"], keep_paths=True)
    got = fullframe.digest(out["paths"], out["rays"])
    res = fullframe.compare(got, want)
    res["stats_world_rays"] = out["stats"]["world_rays"]
    print(name, res)
    if res["hash_mismatch_groups"] or res["ray_mismatch_groups"]:
        g = want["group"]
        bad_groups = np.flatnonzero(fullframe.fold(got, g)["ghash"] != want["ghash"])
        _save_diag(name, (bad_groups[:, None] * g + np.arange(g)[None, :]).ravel(), out)
    assert out["stats"]["world_rays"] == m["world_rays"], res
    assert res["ray_mismatch_groups"] == 0 and res["hash_mismatch_groups"] == 0, res


@pytest.mark.parametrize("name", ["c3_full", "c3m_full"])
def test_c3_full_frame_is_the_reference_frame(name):
    """C3's WHOLE 512x512x1024 frame (268 M paths): the microfacet teapot
    (beckmann 0.01 / 0.05, Raytracing_n.cpp:324, material.h:151-199,
    microfacet_distribution.h) and the dielectric sphere (material.h:282-325), and
    the metal-teapot variant (:348); per-pixel world rays, path hashes and means
    against the reference's own render (tests/golden/make_fullframe.py)."""
    m = fullframe.meta(name)
    want = fullframe.load(name)
    out = capi.Renderer(fullframe.scene_text(name)).render(m["nx"], m["ny"], m["spp"], m["max_depth"], keep_paths=True)
    got = fullframe.digest(out["paths"], out["rays"])
    got["mean"] = out["mean"]
    res = fullframe.compare(got, want)
    res["stats_world_rays"] = out["stats"]["world_rays"]
    print(name, res)
    _save_diag(name, np.flatnonzero((got["hash"] != want["hash"]) | (got["rays"] != want["rays"])), out)
    assert out["stats"]["world_rays"] == m["world_rays"], res
    assert res["ray_mismatch_pixels"] == 0 and res["hash_mismatch_pixels"] == 0, res
    assert res["mean_mismatch_pixels"] == 0, res


@pytest.mark.parametrize("name", ["c4_full", "c4r_full"])
def test_1080p_sample_windows_are_the_reference_frame(name, monkeypatch):
    """A 1080p frame cut into sample windows (renderer.cpp paths_enqueue: a window
    holds as many samples of every pixel as SRR_WINDOW_MB allows; the bench's C4
    frame runs 2 per frame): SRR_WINDOW_MB=150 gives windows of 6, 6 and 4 of the
    16 samples, so each pixel's paths come from three k_paths launches and are summed
    across two window boundaries -- every path and every pixel group still the
    reference's."""
    monkeypatch.setenv("SRR_WINDOW_MB", "150")
    m = fullframe.meta(name)
    want = fullframe.load(name)
    out = capi.Renderer(fullframe.scene_text(name)).render(m["nx"], m["ny"], m["spp"], m["max_depth"], keep_paths=True)
    assert out["stats"]["trace_launches"] == 3, out["stats"]
    got = fullframe.digest(out["paths"], out["rays"])
    res = fullframe.compare(got, want)
    print(name, "windows", res)
    assert out["stats"]["world_rays"] == m["world_rays"], res
    assert res["ray_mismatch_groups"] == 0 and res["hash_mismatch_groups"] == 0, res
