"""Per-path parity metrics shared by the GPU tests, smoke() and bench.py.

Tolerance (written here and in DESIGN.md §6): a path matches when
its radiance equals the reference's within 1e-3 relative (|a-b| <= 1e-3 *
max(|a|, |b|) + 1e-6 per channel), NaN matching NaN; >= 99 % of paths must
match (the tolerance SURVEY §8(d) proposes), and -- the bar the GPU tests actually
hold -- every path must be bit-identical (MIN_BITEXACT = 1.0)."""
from __future__ import annotations

import numpy as np

REL_TOL = 1e-3
ABS_TOL = 1e-6
MIN_MATCH = 0.99
MIN_BITEXACT = 1.0  # every path bit-identical (NaN payloads aside): DESIGN.md §2


def compare_paths(got: np.ndarray, want: np.ndarray) -> dict:
    g = got.reshape(-1, 3).astype(np.float64)
    w = want.reshape(-1, 3).astype(np.float64)
    both_nan = np.isnan(g) & np.isnan(w)
    with np.errstate(invalid="ignore"):
        close = np.abs(g - w) <= REL_TOL * np.maximum(np.abs(g), np.abs(w)) + ABS_TOL
    close = close | both_nan | (g == w)
    path_ok = close.all(axis=1)
    # bit-identical per channel; two NaNs count as identical whatever their payload
    # (x86 produces the negative default NaN, gfx950 the positive one)
    bit = ((got.reshape(-1, 3).view(np.uint32) == want.reshape(-1, 3).view(np.uint32)) | both_nan).all(axis=1)
    return dict(paths=int(path_ok.size), match=float(path_ok.mean()), bitexact=float(bit.mean()),
                worst=np.flatnonzero(~path_ok)[:8].tolist())


def compare_images(got_mean: np.ndarray, want_mean: np.ndarray) -> dict:
    g = got_mean.astype(np.float64)
    w = want_mean.astype(np.float64)
    lum_g, lum_w = g.mean(), w.mean()
    return dict(rmse=float(np.sqrt(np.mean((g - w) ** 2))), mean_rel=float(abs(lum_g - lum_w) / max(lum_w, 1e-12)),
                max_abs=float(np.max(np.abs(g - w))))
