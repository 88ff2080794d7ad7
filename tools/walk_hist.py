"""Mesh-walk length distribution per config (run via gpurun from the repo root).

Renders each config once through the engine that counts traversal work
(SRR_FLAG_COUNT_VISITS: the same BVH4 walk, mesh_hit4 with pruning, as k_paths)
and prints the node steps per world ray through the mesh as a histogram
(the renderer's SRR_HIST=1 line, on stderr).  tools/walk_sim.py turns the
histograms into the predicted effect of suspending long walks.

    SRR_HIST=1 python tools/walk_hist.py [spp] 2> gpurun_out/walk_hist.txt
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "simple-raytracing-render_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402,F401

from srr import capi, scenes  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 8
import soldier_fixture  # noqa: E402

cfgs = [("c2", scenes.s2_cornell_teapot()[0].text(), 512, 512), ("c3", scenes.s3_cornell_teapot_microfacet()[0].text(), 512, 512),
        ("c4", scenes.s4_soldier_standin()[0].text(), 1920, 1080), ("c5", scenes.s5_soldier_fog()[0].text(), 1920, 1080),
        ("c4r", soldier_fixture.scene_text(), 1920, 1080)]
only = os.environ.get("WALK_CFGS")
for name, text, nx, ny in cfgs:
    if only and name not in only.split(","):
        continue
    r = capi.Renderer(text)
    print(f"== {name} {nx}x{ny}x{spp}", file=sys.stderr, flush=True)
    st = r.render(nx, ny, spp, 50, flags=capi.FLAG_COUNT_VISITS)["stats"]
    print(f"   world rays {st['world_rays']} box tests {st['box_tests']} tri tests {st['tri_tests']}",
          file=sys.stderr, flush=True)
