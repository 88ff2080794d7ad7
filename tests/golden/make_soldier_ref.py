"""Golden of the reference's real C4 scene at its configured 1920x1080 frame
(C4_real was pinned to the reference only through the restatement):
the REFERENCE's own paths (oracle/_ref/ref_harness paths) of the committed soldier
fixture's scene (tests/soldier_fixture.py) on 400 pixels -- 250 in the window
around the soldier, 150 over the frame -- at 32 samples per pixel.

    python tests/golden/make_soldier_ref.py      (development container: needs the harness)
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")

import soldier_fixture  # noqa: E402

NX, NY, SPP, DEPTH = 1920, 1080, 32, 50


def pixels():
    rng = np.random.default_rng(2024)
    x0, x1, y0, y1 = 700, 1220, 250, 1000  # around the soldier (tests/test_soldier_scene.py)
    win = rng.integers(y0, y1, 250) * NX + rng.integers(x0, x1, 250)
    return np.unique(np.concatenate([rng.choice(NX * NY, 150, replace=False), win])).astype(np.int64)


def main():
    pix = pixels()
    out = os.path.join(HERE, "soldier_1080")
    with tempfile.TemporaryDirectory() as td:
        scene = os.path.join(td, "soldier.scene")
        with open(scene, "w") as f:
            f.write(soldier_fixture.scene_text())
        r = subprocess.run([HARNESS, "paths", scene, str(NX), str(NY), str(SPP), str(DEPTH),
                            ",".join(map(str, pix)), out], check=True, capture_output=True, text=True)
    stats = json.loads(r.stdout.strip().splitlines()[-1])
    meta = {"nx": NX, "ny": NY, "spp": SPP, "max_depth": DEPTH, "pixels": pix.tolist(),
            "world_rays": stats["world_rays"]}
    with open(out + ".json", "w") as f:
        json.dump(meta, f, indent=1)
    print(len(pix), "pixels", stats)


if __name__ == "__main__":
    main()
