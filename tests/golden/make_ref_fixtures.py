"""Fixtures that let the GPU box (where /root/reference is absent) render the
reference-builder goldens tests/golden/refb_* / reft_* (made by the REFERENCE,
tests/golden/make_scenes.py): each scene as srr builds it from the reference's
assets, flattened to its description, with its decoded RGB8 images stored
2-D-differenced and LZMA-compressed (make_soldier.py's packing), one copy per
distinct image.  reft_soldier_scene reuses soldier_scene.npz: the two scenes
differ only in the camera's aspect, so only its camera line is stored.

The large-mesh goldens (reft_cornell_box, reft_teapot_scene,
reft_jadebunny_scene: 16-32 MB of triangles each as text) and refb_random_scene
(six 2048x2048 textures) are not flattened: tests/golden/ref_assets.npz holds the
asset FILES their builders read (bunny.ply LZMA-compressed, sky_2.png, the six
sky_1 JPEGs: the reference's own data files, byte for byte), and
tests/ref_fixtures.py lays them out as a contents/ directory for srr's builders
(srr/ref_scenes.py) on hosts without /root/reference.

    python tests/golden/make_ref_fixtures.py      (development container)
"""
import hashlib
import json
import lzma
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracing-render_amd"))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(HERE))

from make_soldier import pack  # noqa: E402
from srr import ref_scenes  # noqa: E402

OUT = os.path.join(HERE, "ref_scene_fixtures.npz")
ASSETS_OUT = os.path.join(HERE, "ref_assets.npz")
# the files the builders of the remaining goldens read (contents/-relative)
ASSETS = ["models/bunny.ply", "environment_map/sky_2.png"] + [
    f"environment_map/sky_1/{f}.jpg" for f in ("Front", "Back", "Left", "Right", "Top", "Bottom")]


def asset_key(rel: str) -> str:
    return "file_" + rel.replace("/", "__").replace(".", "_dot_")
CONTENTS = "/root/reference/contents"
KEYS = ["refb_ball_scenes", "refb_final", "reft_ball_orennayar_scenes", "reft_flatnormal_bunny"]


def main():
    meta = json.load(open(os.path.join(HERE, "ref_scenes.json")))
    arrays, images = {}, {}
    for key in KEYS:
        m = meta[key]
        text = ref_scenes.BUILDERS[m["builder"]](m["nx"] / m["ny"], CONTENTS, **m["kwargs"]).text()
        out = []
        for line in text.splitlines():
            mm = re.match(r"^(tex \d+ image_raw) (\d+) (\d+) (\S+)$", line)
            if mm:
                w, h, fn = int(mm.group(2)), int(mm.group(3)), mm.group(4)
                raw = np.fromfile(fn, np.uint8).reshape(h, w, 3)
                k = "img_" + hashlib.sha256(raw.tobytes()).hexdigest()[:16]
                images[k] = raw
                line = f"{mm.group(1)} {w} {h} @{k}"
            out.append(line)
        arrays["text_" + key] = np.frombuffer("\n".join(out).encode() + b"\n", np.uint8)
    # reft_soldier_scene: the soldier fixture's scene with this golden's camera line
    m = meta["reft_soldier_scene"]
    small = ref_scenes.soldier_scene(m["nx"] / m["ny"], contents=CONTENTS).text().splitlines()
    big = ref_scenes.soldier_scene(1920 / 1080, contents=CONTENTS).text().splitlines()
    diff = [i for i, (a, b) in enumerate(zip(small, big)) if a != b]
    assert len(small) == len(big) and len(diff) == 1 and small[diff[0]].startswith("camera "), diff
    arrays["camera_reft_soldier_scene"] = np.frombuffer(small[diff[0]].encode(), np.uint8)
    for k, v in images.items():
        arrays[k] = np.frombuffer(pack(v), np.uint8)
        arrays[k + "_shape"] = np.array(v.shape, np.int64)
    np.savez(OUT, **arrays)
    print(OUT, os.path.getsize(OUT), "bytes;", len(images), "images")
    assets = {}
    for rel in ASSETS:
        data = open(os.path.join(CONTENTS, rel), "rb").read()
        if rel.endswith(".ply"):
            data = lzma.compress(data, preset=9 | lzma.PRESET_EXTREME)
        assets[asset_key(rel)] = np.frombuffer(data, np.uint8)
    np.savez(ASSETS_OUT, **assets)
    print(ASSETS_OUT, os.path.getsize(ASSETS_OUT), "bytes;", len(assets), "asset files")


if __name__ == "__main__":
    main()
