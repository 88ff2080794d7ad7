"""Golden renders of the reference's own scene builders (Raytracing_n.cpp:108-711)
made by the REFERENCE's code (oracle/_ref/ref_harness; development container
only, needs /root/reference):

    python tests/golden/make_scenes.py

Two kinds, both per-path radiance + world-ray counts (same layout as
make_golden.py's renders), at small sizes:

* ``refb_<name>``: the reference's builder FUNCTION itself (harness `builder`),
  run in a scratch directory holding the literal Windows asset paths it opens
  ("..\\contents\\...") as links to /root/reference/contents.  This pins
  srr/ref_scenes.py's restatement of the builder -- constructor order, every
  drand48() draw, asset decoding -- not just the renderer.  Available for the
  builders that need no assimp model: random_scene, ball_scenes, final.
* ``reft_<name>``: the scene text srr/ref_scenes.py emits, built into the
  REFERENCE's classes by the harness (`render`): the builders that load models
  (assimp is Win32-only here) and ball_orennayar_scenes, whose
  builder overflows its 21-slot list with 24 objects (Raytracing_n.cpp:438) and
  crashes.
"""
from __future__ import annotations

import glob
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracing-render_amd"))

from srr import ref_scenes  # noqa: E402

REF = "/root/reference"
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")

# (name, kind, nx, ny, spp, builder kwargs)
RENDERS = [
    ("random_scene", "b", 16, 12, 4, {}),
    ("ball_scenes", "b", 16, 12, 4, {}),
    ("final", "b", 16, 12, 4, {}),
    ("ball_orennayar_scenes", "t", 16, 12, 4, {}),
    ("cornell_box", "t", 16, 12, 4, {}),
    ("jadebunny_scene", "t", 16, 12, 4, {}),
    ("soldier_scene", "t", 16, 12, 4, {}),
    ("flatnormal_bunny", "t", 16, 12, 4, {}),
    ("teapot_scene", "t", 12, 9, 2, {}),
]


def link_contents(td):
    for f in glob.glob(os.path.join(REF, "contents", "**", "*"), recursive=True):
        if os.path.isfile(f):
            name = "..\\" + os.path.relpath(f, REF).replace("/", "\\")
            os.symlink(f, os.path.join(td, name))


def main():
    meta = {}
    with tempfile.TemporaryDirectory() as td:
        link_contents(td)
        for name, kind, nx, ny, spp, kw in RENDERS:
            out = os.path.join(HERE, f"ref{kind}_{name}")
            if kind == "b":
                cmd = [HARNESS, "builder", name, str(nx), str(ny), str(spp), "50", out]
            else:
                text = ref_scenes.BUILDERS[name](nx / ny, **kw).text()
                sp = os.path.join(td, f"{name}.scene")
                open(sp, "w").write(text)
                cmd = [HARNESS, "render", sp, str(nx), str(ny), str(spp), "50", out]
            r = subprocess.run(cmd, cwd=td, capture_output=True, text=True, check=True)
            stats = json.loads(r.stdout.strip().splitlines()[-1])
            for ext in (".img.f32", ".ppm"):
                if os.path.exists(out + ext):
                    os.remove(out + ext)
            meta[f"ref{kind}_{name}"] = dict(builder=name, kind=kind, nx=nx, ny=ny, spp=spp, max_depth=50,
                                             kwargs=kw, world_rays=stats["world_rays"])
            print(name, kind, stats)
    with open(os.path.join(HERE, "ref_scenes.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
