"""Scene texts of the reference-builder goldens (tests/golden/refb_* / reft_*) for
hosts without /root/reference: tests/golden/ref_scene_fixtures.npz (made by
tests/golden/make_ref_fixtures.py) with its images restored to raw RGB8 files
under a temporary directory, and reft_soldier_scene from the soldier fixture
with that golden's camera line."""
import os
import tempfile

import numpy as np

import soldier_fixture

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_scene_fixtures.npz")
KEYS = ["refb_ball_scenes", "refb_final", "reft_ball_orennayar_scenes", "reft_flatnormal_bunny", "reft_soldier_scene"]
_DIR = None


def scene_text(key: str) -> str:
    global _DIR
    z = np.load(FIXTURE)  # plain arrays only (allow_pickle stays False)
    if key == "reft_soldier_scene":
        cam = z["camera_reft_soldier_scene"].tobytes().decode()
        lines = soldier_fixture.scene_text().splitlines()
        i = next(i for i, l in enumerate(lines) if l.startswith("camera "))
        lines[i] = cam
        return "\n".join(lines) + "\n"
    if _DIR is None:
        _DIR = tempfile.mkdtemp(prefix="srr_refscenes_")
    lines = []
    for line in z["text_" + key].tobytes().decode().splitlines():
        if " @img_" in line:
            head, k = line.rsplit(" @", 1)
            fn = os.path.join(_DIR, k + ".rgb")
            if not os.path.exists(fn):
                soldier_fixture.unpack(z[k].tobytes(), tuple(z[k + "_shape"])).tofile(fn)
            line = f"{head} {fn}"
        lines.append(line)
    return "\n".join(lines) + "\n"
