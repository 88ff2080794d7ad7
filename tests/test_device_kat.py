"""Device known-answer tests: the HIP implementations of the reference's
per-function code (material.h, pdf.h, microfacet_distribution.h, common.h,
triangle.h, aabb.h, camera.h, light sampling of aarect.h / sphere.h / triangle.h /
hitable_list.h), run through srr_device_kat on the reference's own KAT
records (tests/golden/kat_*.bin, made by oracle/ref from the reference's
functions), must reproduce the reference's outputs bit for bit."""
import ctypes

import numpy as np
import pytest

import oracle_bind as ob
from srr import capi

# output columns per KAT (inputs come first; oracle/ref/kat.inc layouts)
OUT = {"erf": range(1, 3), "beckmann11": range(3, 5), "beckmann_dist": range(7, 16),
       "beckmann_pdf": range(12, 21), "cosine_pdf": list(range(9, 16)) + [19, 20],
       "orennayar_pdf": list(range(9, 16)) + [19, 20], "dielectric": range(9, 14), "metal": range(9, 14),
       "triangle": range(16, 26), "aabb": [14], "camera": range(14, 23), "lights": range(5, 15),
       "light_list": range(5, 15)}


def device_kat(name, rec):
    L = capi.lib()
    L.srr_device_kat.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    out = np.ascontiguousarray(rec.copy())
    capi._check(L.srr_device_kat(name.encode(), out.shape[0], out.shape[1], out.ctypes.data))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(OUT))
def test_device_kat_bitexact(name):
    rec = ob.read_kat(name)
    got = device_kat(name, rec)
    cols = list(OUT[name])
    g = got[:, cols].view(np.uint32)
    w = rec[:, cols].view(np.uint32)
    eq = (g == w) | (np.isnan(got[:, cols]) & np.isnan(rec[:, cols]))
    if name == "triangle":  # a medium ray's back-face hit: the record re-test is front-only (hit and t only)
        back = (rec[:, 15] != 0)
        eq[back, 2:] = True
    bad = np.flatnonzero(~eq.all(axis=1))
    per_col = {c: int((~eq[:, k]).sum()) for k, c in enumerate(cols) if (~eq[:, k]).any()}
    for i in bad[:4]:
        print(name, "record", i, "in", rec[i, :cols[0]].tolist(), "\n  ref", rec[i, cols].tolist(),
              "\n  dev", got[i, cols].tolist())
    assert len(bad) == 0, f"{name}: {len(bad)} of {len(rec)} records differ; per output column {per_col}"


@pytest.mark.gpu
def test_device_sqrt_correctly_rounded():
    """The device sqrt behind every length / unit_vector rounds like the host's
    sqrtf (correctly rounded), including tiny, huge and exact-square inputs."""
    rng = np.random.default_rng(3)
    bits = rng.integers(0, 0x7F800000, size=2_000_000, dtype=np.int64).astype(np.uint32)
    x = np.concatenate([bits.view(np.float32), np.float32([0, 1, 4, 2, 0.25, 1e-45, 3e38, np.inf]),
                        (np.arange(1, 4097, dtype=np.float32) ** 2)])
    rec = np.stack([x, np.zeros_like(x)], 1).astype(np.float32)
    got = device_kat("sqrt", rec)[:, 1]
    want = np.sqrt(x.astype(np.float32))
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
