"""Fixture of the reference's real C4 scene, soldier_scene (Raytracing_n.cpp:585-657,
sceneid 6), for the GPU box (where /root/reference is absent): the scene as srr
builds it from the reference's own assets (srr/ref_scenes.py soldier_scene: the
Soilder.FBX mesh 0 through srr's binary-FBX loader -- assimp replaced, parity
against assimp unpinned --, sky4.jpg and the two PNG textures through srr's
stb-exact decoder), flattened to its scene description with explicit triangles,
plus the three decoded RGB8 images.  Images are stored 2-D-differenced (mod 256)
and LZMA-compressed: tests/soldier_fixture.py restores them bit for bit.

    python tests/golden/make_soldier.py      (development container)
"""
import lzma
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracing-render_amd"))

from srr import ref_scenes  # noqa: E402

OUT = os.path.join(HERE, "soldier_scene.npz")
ASPECT = 1920 / 1080


def pack(rgb: np.ndarray) -> bytes:
    d = rgb.astype(np.uint8)
    d = np.diff(d, axis=1, prepend=np.uint8(0)).astype(np.uint8)  # left differences
    d = np.diff(d, axis=0, prepend=np.uint8(0)).astype(np.uint8)  # then up differences
    return lzma.compress(d.tobytes(), preset=6)


def main():
    text = ref_scenes.soldier_scene(ASPECT, contents="/root/reference/contents").text()
    out, images = [], {}
    for line in text.splitlines():
        m = re.match(r"^(tex \d+ image_raw) (\d+) (\d+) (\S+)$", line)
        if m:
            w, h, fn = int(m.group(2)), int(m.group(3)), m.group(4)
            key = f"img{len(images)}"
            raw = np.fromfile(fn, np.uint8).reshape(h, w, 3)
            images[key] = raw
            line = f"{m.group(1)} {w} {h} @{key}"
        out.append(line)
    arrays = {"text": np.frombuffer("\n".join(out).encode() + b"\n", np.uint8)}
    for k, v in images.items():
        arrays[k] = np.frombuffer(pack(v), np.uint8)
        arrays[k + "_shape"] = np.array(v.shape, np.int32)
    np.savez(OUT, **arrays)
    print(OUT, os.path.getsize(OUT), {k: v.shape for k, v in images.items()}, len(out), "lines")


if __name__ == "__main__":
    main()
