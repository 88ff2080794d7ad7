"""Progressive rendering with resume.

The reference renders a frame in one pass (Raytracing_n.cpp:815-879).  Here a
frame can be built up in chunks of samples -- each a render of the next sample
range [samples, samples + n) with SRR_FLAG_CONTINUE, added to the renderer's
per-pixel running sums in sample order -- and its state saved and resumed in
another process.  Per-path seeds and Sobol points depend only on (pixel, global
sample index), so any chunking gives bitwise the image of one render of all the
samples (tests/test_progressive.py).
"""
from __future__ import annotations

import ctypes
import hashlib

import numpy as np

from . import capi


class Progressive:
    def __init__(self, renderer: "capi.Renderer", nx: int, ny: int, max_depth: int = 50, flags: int = 0, **params):
        self.r = renderer
        self.nx, self.ny, self.max_depth = nx, ny, max_depth
        self.flags = flags  # engine flags (e.g. capi.FLAG_WAVEFRONT)
        self.params = params  # shard / tile / base_seed ... (capi.make_params keywords)
        self.samples = 0
        self.mean = None

    def step(self, spp: int) -> np.ndarray:
        """Render the next `spp` samples of every pixel; returns the mean over all
        samples so far (before the reference's sqrt / 8-bit tone map)."""
        flags = self.flags | (capi.FLAG_CONTINUE if self.samples else 0)
        out = self.r.render(self.nx, self.ny, spp, self.max_depth, sample_begin=self.samples, flags=flags,
                            **self.params)
        self.samples += spp
        self.mean = out["mean"]
        return self.mean

    def image8(self) -> np.ndarray:
        return capi.tonemap(self.mean)

    # ------------------------------------------------------------ resume
    def _scene_key(self) -> str:
        text = getattr(self.r.scene, "text", None)
        return hashlib.sha256(text.encode()).hexdigest() if isinstance(text, str) else ""

    def save(self, path: str) -> None:
        """Per-pixel running sums + sample count + frame parameters (.npz)."""
        L = capi.lib()
        npix, samples = ctypes.c_int64(), ctypes.c_int64()
        capi._check(L.srr_accum_get(self.r.h, None, ctypes.byref(npix), ctypes.byref(samples)))
        sums = np.zeros((npix.value, 3), np.float32)
        capi._check(L.srr_accum_get(self.r.h, capi._ptr(sums), None, None))
        np.savez(path, sums=sums, samples=samples.value, nx=self.nx, ny=self.ny, max_depth=self.max_depth,
                 scene=self._scene_key())

    def load(self, path: str) -> None:
        """Restore a saved state into this renderer (same scene and frame)."""
        z = np.load(path, allow_pickle=False)
        if (int(z["nx"]), int(z["ny"]), int(z["max_depth"])) != (self.nx, self.ny, self.max_depth):
            raise capi.SrrError("saved state is for a different frame")
        key = self._scene_key()
        if key and str(z["scene"]) and str(z["scene"]) != key:
            raise capi.SrrError("saved state is for a different scene")
        sums = np.ascontiguousarray(z["sums"], np.float32)
        capi._check(capi.lib().srr_accum_set(self.r.h, capi._ptr(sums), sums.shape[0], int(z["samples"])))
        self.samples = int(z["samples"])
