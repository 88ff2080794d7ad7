"""The reference's real C4 scene (soldier_scene, Raytracing_n.cpp:585-657) from its
committed fixture (tests/golden/make_soldier.py): scene_text() returns the srr
scene description with the three images restored to raw RGB8 files under a
temporary directory.  Used by the GPU tests and bench.py --scene s4_real."""
import lzma
import os
import tempfile

import numpy as np

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "soldier_scene.npz")
_TEXT = None


def require(path: str) -> None:
    """The reference-asset fixtures (THIRD_PARTY_NOTICES.md) may be deleted by a
    redistributor: a test that needs an absent one is skipped, anything else fails."""
    if os.path.exists(path):
        return
    msg = f"{os.path.basename(path)} absent (a reference-asset fixture, THIRD_PARTY_NOTICES.md)"
    if "PYTEST_CURRENT_TEST" in os.environ:
        import pytest
        pytest.skip(msg)
    raise FileNotFoundError(msg)


def unpack(blob: bytes, shape) -> np.ndarray:
    d = np.frombuffer(lzma.decompress(blob), np.uint8).reshape(shape)
    d = np.cumsum(d, axis=0, dtype=np.uint8)  # undo the up differences (mod 256)
    return np.cumsum(d, axis=1, dtype=np.uint8)  # then the left differences


def scene_text() -> str:
    global _TEXT
    if _TEXT is None:
        require(FIXTURE)
        z = np.load(FIXTURE)  # plain arrays only (allow_pickle stays False)
        d = tempfile.mkdtemp(prefix="srr_soldier_")
        lines = []
        for line in z["text"].tobytes().decode().splitlines():
            if " @img" in line:
                head, key = line.rsplit(" @", 1)
                fn = os.path.join(d, key + ".rgb")
                unpack(z[key].tobytes(), tuple(z[key + "_shape"])).tofile(fn)
                line = f"{head} {fn}"
            lines.append(line)
        _TEXT = "\n".join(lines) + "\n"
    return _TEXT
