"""ctypes binding of oracle/liboracle.so (the CPU restatement).  Test
infrastructure: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it, and only as the checker / CPU baseline."""
from __future__ import annotations

import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(ROOT, "oracle", "liboracle.so")
        if not os.path.exists(path):
            import subprocess
            subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"], check=True,
                           capture_output=True)
        L = ctypes.CDLL(path)
        L.oracle_render.restype = ctypes.c_int
        L.oracle_render.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
        L.oracle_kat.restype = ctypes.c_int
        L.oracle_kat.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_sobol.argtypes = [ctypes.c_int, ctypes.c_void_p]
        L.oracle_teapot.argtypes = [ctypes.c_float, ctypes.c_int, ctypes.c_void_p]
        _LIB = L
    return _LIB


def _p(a):
    return None if a is None else a.ctypes.data


def render(scene_text: str, nx: int, ny: int, spp: int, max_depth: int = 50, pixels=None, threads: int = 1,
           want_paths: bool = True):
    """Returns dict(paths[n,spp,3], rays[n,spp], img[n,3], img8[n,3], stats[5]).

    stats: world rays, box tests, triangle tests, analytic primitive tests,
    resampling loops stopped by the attempt cap."""
    n = nx * ny if pixels is None else len(pixels)
    pix = None if pixels is None else np.ascontiguousarray(pixels, dtype=np.int32)
    paths = np.zeros((n, spp, 3), np.float32) if want_paths else None
    rays = np.zeros((n, spp), np.uint8)
    img = np.zeros((n, 3), np.float32)
    img8 = np.zeros((n, 3), np.uint8)
    stats = np.zeros(5, np.int64)
    rc = lib().oracle_render(scene_text.encode(), nx, ny, spp, max_depth, _p(pix), n, _p(paths), _p(rays), _p(img),
                             _p(img8), _p(stats), threads)
    if rc != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return dict(paths=paths, rays=rays, img=img, img8=img8, stats=stats)


def read_kat(name: str):
    raw = np.fromfile(os.path.join(GOLDEN, f"kat_{name}.bin"), dtype=np.int32, count=2)
    n, w = int(raw[0]), int(raw[1])
    rec = np.fromfile(os.path.join(GOLDEN, f"kat_{name}.bin"), dtype=np.float32, offset=8).reshape(n, w)
    return rec


def replay_kat(name: str, rec: np.ndarray) -> np.ndarray:
    out = np.ascontiguousarray(rec.copy())
    rc = lib().oracle_kat(name.encode(), out.shape[0], out.shape[1], _p(out))
    if rc != 0:
        raise RuntimeError(lib().oracle_last_error().decode())
    return out


def sobol(n: int) -> np.ndarray:
    out = np.zeros((n, 2), np.float64)
    lib().oracle_sobol(n, _p(out))
    return out


def teapot(scale: float, divs: int) -> np.ndarray:
    out = np.zeros((32 * divs * divs * 2, 12), np.float32)
    lib().oracle_teapot(scale, divs, _p(out))
    return out
