"""Scene texts of the reference-builder goldens (tests/golden/refb_* / reft_*) for
hosts without /root/reference: tests/golden/ref_scene_fixtures.npz (made by
tests/golden/make_ref_fixtures.py) with its images restored to raw RGB8 files
under a temporary directory, reft_soldier_scene from the soldier fixture with
that golden's camera line, and the large-mesh / large-texture goldens built by
srr's builders from the reference's asset files (tests/golden/ref_assets.npz)."""
import os
import tempfile

import numpy as np

import soldier_fixture

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_scene_fixtures.npz")
ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_assets.npz")
# goldens whose flattened scene is stored (ref_scene_fixtures.npz) ...
TEXT_KEYS = ["refb_ball_scenes", "refb_final", "reft_ball_orennayar_scenes", "reft_flatnormal_bunny",
             "reft_soldier_scene"]
# ... and goldens whose builders run on the stored asset files (ref_assets.npz)
BUILDER_KEYS = ["reft_cornell_box", "reft_teapot_scene", "reft_jadebunny_scene", "refb_random_scene"]
KEYS = TEXT_KEYS + BUILDER_KEYS
_DIR = None
_CONTENTS = None


def contents_dir() -> str:
    """The reference's asset files the BUILDER_KEYS scenes read, laid out as its
    contents/ directory in a temporary directory (bunny.ply decompressed)."""
    import lzma
    global _CONTENTS
    if _CONTENTS is None:
        soldier_fixture.require(ASSETS)
        d = tempfile.mkdtemp(prefix="srr_contents_")
        z = np.load(ASSETS)  # plain arrays only (allow_pickle stays False)
        for k in z.files:
            rel = k[len("file_"):].replace("__", "/").replace("_dot_", ".")
            data = z[k].tobytes()
            if rel.endswith(".ply"):
                data = lzma.decompress(data)
            os.makedirs(os.path.join(d, os.path.dirname(rel)), exist_ok=True)
            with open(os.path.join(d, rel), "wb") as f:
                f.write(data)
        _CONTENTS = d
    return _CONTENTS


def scene_text(key: str) -> str:
    global _DIR
    if key in BUILDER_KEYS:
        import json

        from srr import ref_scenes
        m = json.load(open(os.path.join(os.path.dirname(FIXTURE), "ref_scenes.json")))[key]
        return ref_scenes.BUILDERS[m["builder"]](m["nx"] / m["ny"], contents_dir(), **m["kwargs"]).text()
    soldier_fixture.require(FIXTURE)
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
