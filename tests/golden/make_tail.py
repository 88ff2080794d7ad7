"""Golden for the C2 frame's tail rays: every path of the
12 pixels of the full 512x512x1024 C2 frame whose paths contain a world ray
with a NaN t bound -- a ray leaving a wall point at y = 554 exactly toward the
ceiling light, which lies in the light's plane: the light's xz_rect::hit
returns t = (554 - 554) / 0 = NaN (aarect.h:113-129), so closest_so_far is NaN
when the teapot is tested and the reference walks its whole BVH
(aabb.h:33-49 rejects no box).  Before round 3 each such ray cost the GPU 8-17
ms (kernels.hip mesh_scan_nan).  The pixels were captured on the GPU by the
diagnostics build (tools/slow_rays.py, profiles/r03/nan_bound_rays_s2.jsonl);
their paths here are the REFERENCE's own (oracle/_ref/ref_harness paths).

    python tests/golden/make_tail.py      (development container: needs the harness)
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")

# (pixel, sample) of each captured NaN-bound ray, PPM-order pixel index
CAPTURED = [(7694, 273), (7667, 587), (11285, 214), (18909, 123), (20442, 315), (22996, 918), (37815, 212),
            (37815, 738), (43091, 753), (43436, 681), (47708, 811), (49569, 559), (55700, 817)]


def main():
    pixels = sorted({p for p, _ in CAPTURED})
    scene = os.path.join(HERE, "c2_full.scene")
    out = os.path.join(HERE, "c2_tail")
    r = subprocess.run([HARNESS, "paths", scene, "512", "512", "1024", "50", ",".join(map(str, pixels)), out],
                       check=True, capture_output=True, text=True)
    stats = json.loads(r.stdout.strip().splitlines()[-1])
    meta = {"scene": "c2_full.scene", "nx": 512, "ny": 512, "spp": 1024, "max_depth": 50, "pixels": pixels,
            "captured": CAPTURED, "world_rays": stats["world_rays"]}
    with open(out + ".json", "w") as f:
        json.dump(meta, f, indent=1)
    print(meta)


if __name__ == "__main__":
    main()
