"""The full-frame digest format (tests/fullframe.py) against the reference:
the digest of the s2 golden's per-path outputs (made by the reference's own
renderer) equals the reference's own per-pixel digest of the same frame
(`ref_harness sums`), and the CPU restatement reproduces both."""
import numpy as np

import fullframe
import oracle_bind as ob


def test_digest_of_golden_paths_matches_reference_digest():
    import json
    m = json.load(open(f"{ob.GOLDEN}/golden.json"))["renders"]["s2"]
    n = m["nx"] * m["ny"]
    paths = np.fromfile(f"{ob.GOLDEN}/s2.paths.f32", np.float32).reshape(n, m["spp"], 3)
    rays = np.fromfile(f"{ob.GOLDEN}/s2.rays.u8", np.uint8).reshape(n, m["spp"])
    img = np.fromfile(f"{ob.GOLDEN}/s2.img.f32", np.float32).reshape(n, 3)
    want = fullframe.load("s2_digest")
    got = fullframe.digest(paths, rays)
    got["mean"] = img
    res = fullframe.compare(got, want)
    assert res["hash_mismatch_pixels"] == 0 and res["ray_mismatch_pixels"] == 0, res
    assert res["mean_mismatch_pixels"] == 0, res
    assert res["world_rays"] == fullframe.meta("s2_digest")["world_rays"] == m["world_rays"]


def test_digest_detects_one_changed_path():
    want = fullframe.load("s2_digest")
    m = fullframe.meta("s2_digest")
    n = m["nx"] * m["ny"]
    paths = np.fromfile(f"{ob.GOLDEN}/s2.paths.f32", np.float32).reshape(n, m["spp"], 3).copy()
    rays = np.fromfile(f"{ob.GOLDEN}/s2.rays.u8", np.uint8).reshape(n, m["spp"]).copy()
    paths[77, 5, 1] = np.nextafter(paths[77, 5, 1], np.float32(np.inf))
    rays[300, 9] += 1
    res = fullframe.compare(fullframe.digest(paths, rays), want)
    assert res["hash_mismatch_pixels"] == 2 and res["ray_mismatch_pixels"] == 1, res
    assert res["first_bad"] == [77, 300]


def test_restatement_reproduces_c2_full_frame_rows():
    """The CPU restatement on two full rows of the headline C2 frame (512 pixels
    x 1024 samples each) against the reference's full-frame digest."""
    m = fullframe.meta("c2_full")
    want = fullframe.load("c2_full")
    nx = m["nx"]
    rows = [3, 300]
    pix = np.concatenate([np.arange(r * nx, (r + 1) * nx) for r in rows]).astype(np.int32)
    out = ob.render(fullframe.scene_text("c2_full"), m["nx"], m["ny"], m["spp"], m["max_depth"], pixels=pix,
                    threads=8)
    got = fullframe.digest(out["paths"], out["rays"])
    got["mean"] = out["img"]
    res = fullframe.compare(got, {k: v[pix] for k, v in want.items()})
    assert res["hash_mismatch_pixels"] == 0 and res["mean_mismatch_pixels"] == 0, res


def test_fold_detects_one_changed_path_in_a_group():
    m = fullframe.meta("s2_digest")
    n = m["nx"] * m["ny"]
    paths = np.fromfile(f"{ob.GOLDEN}/s2.paths.f32", np.float32).reshape(n, m["spp"], 3).copy()
    rays = np.fromfile(f"{ob.GOLDEN}/s2.rays.u8", np.uint8).reshape(n, m["spp"]).copy()
    want = fullframe.fold(fullframe.digest(paths, rays), 16)
    paths[77, 5, 1] = np.nextafter(paths[77, 5, 1], np.float32(np.inf))
    res = fullframe.compare(fullframe.digest(paths, rays), want)
    assert res["hash_mismatch_groups"] == 1 and res["ray_mismatch_groups"] == 0 and res["first_bad_group"] == [4]


import pytest  # noqa: E402


@pytest.mark.parametrize("name", ["c4_full", "c5_full", "c4r_full"])
def test_restatement_reproduces_1080p_full_frame_groups(name):
    """The CPU restatement on 48 pixel groups (768 pixels x 16 samples) of each
    1920x1080 reference frame (C4 / C5 stand-ins, C4_real) against the
    reference's grouped digests."""
    m = fullframe.meta(name)
    want = fullframe.load(name)
    g = want["group"]
    groups = np.linspace(0, want["grays"].size - 1, 48).astype(np.int64)
    pix = (groups[:, None] * g + np.arange(g)[None, :]).ravel().astype(np.int32)
    out = ob.render(fullframe.scene_text(name), m["nx"], m["ny"], m["spp"], m["max_depth"], pixels=pix, threads=8)
    got = fullframe.fold(fullframe.digest(out["paths"], out["rays"]), g)
    assert np.array_equal(got["grays"], want["grays"][groups])
    assert np.array_equal(got["ghash"], want["ghash"][groups])
