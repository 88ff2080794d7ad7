"""Per-pixel digests of a full frame (the format tests/golden/make_fullframe.py
writes from the reference's own renderer): world-ray sums, a word-wise FNV-1a-32
over every path's (r, g, b, rays) in sample order with NaNs canonicalised, and
the mean radiance.  Test infrastructure only."""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")
FNV_OFFSET = np.uint32(2166136261)
FNV_PRIME = np.uint32(16777619)
CANON_NAN = np.uint32(0x7FC00000)


def meta(name: str) -> dict:
    return json.load(open(os.path.join(GOLDEN, "fullframe.json")))[name]


def load(name: str) -> dict:
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    if "group" in z.files:  # digests folded over runs of `group` pixels (fold)
        return dict(grays=z["grays"], ghash=z["ghash"], group=int(z["group"]))
    return dict(rays=z["rays"], hash=z["hash"], mean=z["mean"])


def scene_text(name: str) -> str:
    path = os.path.join(GOLDEN, f"{name}.scene")
    if os.path.exists(path):
        return open(path).read()
    if name == "c4r_full":  # the soldier fixture's scene (its images are restored to temp files)
        import soldier_fixture
        return soldier_fixture.scene_text()
    raise FileNotFoundError(path)


def fold(d: dict, group: int) -> dict:
    """Per-pixel digests folded over runs of `group` consecutive pixels (PPM
    order): world-ray sums, and a word-wise FNV-1a-32 over the pixels' hashes."""
    rays = d["rays"].reshape(-1, group)
    hs = d["hash"].reshape(-1, group)
    h = np.full(rays.shape[0], FNV_OFFSET, np.uint32)
    for k in range(group):
        h = (h ^ hs[:, k]) * FNV_PRIME
    return dict(grays=rays.sum(axis=1, dtype=np.uint64).astype(np.uint32), ghash=h, group=group)


def digest(paths: np.ndarray, rays: np.ndarray, chunk: int = 2048) -> dict:
    """paths [npix, spp, 3] float32 (raw radiance, before de_nan), rays [npix, spp]."""
    npix, spp = rays.shape
    out_rays = np.empty(npix, np.uint32)
    out_hash = np.empty(npix, np.uint32)
    for a in range(0, npix, chunk):
        b = min(npix, a + chunk)
        p = paths[a:b]
        bits = p.view(np.uint32).copy()
        bits[np.isnan(p)] = CANON_NAN
        bits = np.ascontiguousarray(bits.transpose(1, 2, 0))  # [spp, 3, n]
        r = np.ascontiguousarray(rays[a:b].T).astype(np.uint32)  # [spp, n]
        h = np.full(b - a, FNV_OFFSET, np.uint32)
        for s in range(spp):
            for c in range(3):
                h = (h ^ bits[s, c]) * FNV_PRIME
            h = (h ^ r[s]) * FNV_PRIME
        out_hash[a:b] = h
        out_rays[a:b] = r.sum(axis=0, dtype=np.uint64).astype(np.uint32)
    return dict(rays=out_rays, hash=out_hash)


def compare(got: dict, want: dict) -> dict:
    if "group" in want:
        g = fold(got, want["group"])
        bad_rays = np.flatnonzero(g["grays"] != want["grays"])
        bad_hash = np.flatnonzero(g["ghash"] != want["ghash"])
        return dict(pixels=int(want["grays"].size * want["group"]), groups=int(want["grays"].size),
                    world_rays=int(got["rays"].sum(dtype=np.int64)),
                    want_world_rays=int(want["grays"].sum(dtype=np.int64)), ray_mismatch_groups=int(bad_rays.size),
                    hash_mismatch_groups=int(bad_hash.size), first_bad_group=bad_hash[:16].tolist())
    bad_rays = np.flatnonzero(got["rays"] != want["rays"])
    bad_hash = np.flatnonzero(got["hash"] != want["hash"])
    res = dict(pixels=int(want["rays"].size), world_rays=int(got["rays"].sum(dtype=np.int64)),
               want_world_rays=int(want["rays"].sum(dtype=np.int64)), ray_mismatch_pixels=int(bad_rays.size),
               hash_mismatch_pixels=int(bad_hash.size), first_bad=bad_hash[:16].tolist())
    if "mean" in got:
        g, w = got["mean"].view(np.uint32), want["mean"].view(np.uint32)
        both_nan = np.isnan(got["mean"]) & np.isnan(want["mean"])
        res["mean_mismatch_pixels"] = int((~((g == w) | both_nan)).any(axis=1).sum())
    return res
