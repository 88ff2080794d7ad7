"""Golden decodes of every image the reference ships, made by the REFERENCE's
own stbi_load (stb_image v2.19 compiled inside Raytracing_n.cpp by
oracle/ref's harness; development container only):

    python tests/golden/make_images.py

Writes tests/golden/images.json: per file (path relative to the reference's
root) and req_comp, the decoded size, the channel count stbi_load reports and
the CRC-32 + SHA-256 of the returned bytes.  The images themselves stay in the
reference; tests/test_imageio.py decodes them with srr's decoder (when they are
present) and compares against these digests.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import subprocess
import tempfile
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
EXT = (".png", ".jpg", ".tga", ".bmp")
# extra channel requests, exercised on one file per format
REQ = {"contents/environment_map/sky4.jpg": (1, 2, 4), "contents/textures/earthmap.jpg": (1, 4),
       "contents/textures/Checkerboard.png": (1, 4), "contents/textures/NPC_ChaoJiBing_M.tga": (3,),
       "welcom.bmp": (4,)}


def main():
    files = sorted(os.path.relpath(f, REF) for f in glob.glob(os.path.join(REF, "**", "*"), recursive=True)
                   if f.lower().endswith(EXT))
    out = {}
    with tempfile.TemporaryDirectory() as td:
        raw = os.path.join(td, "img.raw")
        for rel in files:
            for req in (0,) + REQ.get(rel, ()):
                r = subprocess.run([HARNESS, "image", os.path.join(REF, rel), str(req), raw],
                                   capture_output=True, text=True, check=True)
                x, y, n = (int(v) for v in r.stdout.split())
                b = open(raw, "rb").read()
                out[f"{rel}|{req}"] = {"x": x, "y": y, "comp": n, "bytes": len(b),
                                       "crc32": zlib.crc32(b) & 0xFFFFFFFF, "sha256": hashlib.sha256(b).hexdigest()}
                print(rel, req, x, y, n)
    with open(os.path.join(HERE, "images.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
