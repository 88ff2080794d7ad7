"""Fixtures that let the GPU box (where /root/reference is absent) render the
reference-builder goldens tests/golden/refb_* / reft_* (made by the REFERENCE,
tests/golden/make_scenes.py): each scene as srr builds it from the reference's
assets, flattened to its description, with its decoded RGB8 images stored
2-D-differenced and LZMA-compressed (make_soldier.py's packing), one copy per
distinct image.  reft_soldier_scene reuses soldier_scene.npz: the two scenes
differ only in the camera's aspect, so only its camera line is stored.

The large-mesh goldens (reft_cornell_box, reft_teapot_scene,
reft_jadebunny_scene: 16-32 MB of triangles each) and refb_random_scene (six
2048x2048 textures) stay CPU-only.

    python tests/golden/make_ref_fixtures.py      (development container)
"""
import hashlib
import json
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


if __name__ == "__main__":
    main()
