"""The reference's program, ``main()`` (Raytracing_n.cpp:882-952), over srr:
pick a scene by ``sceneid``, build it with the reference's builder (restated in
srr/ref_scenes.py, pinned to the reference's own builder code by
tests/test_ref_builders_compile.py), render nx x ny x ns with maxDepth on the
GPU, print the elapsed milliseconds and write the P3 PPM (the tone map and byte
format of Raytracing_n.cpp:850-886).

    python -m srr.render_main [--sceneid 2] [--nx 1000] [--ny 1000] [--ns 50] [--max-depth 50] [--out out.ppm]
                              [--gpus N]   (srr_renderer_create_multi: one RCCL gather at frame end)

Defaults are the reference's globals (Raytracing_n.cpp:39-43).  Differences, all
forced by the reference: its 8 render threads race on shared state
and its pixel mapping scrambles non-square frames (Q12); srr renders every
(pixel, sample) path with its per-path seed and writes the intended image.
Assets are read from $SRR_CONTENTS (default /root/reference/contents), which
the builders need (images, meshes)."""
from __future__ import annotations

import argparse
import sys
import time

from . import capi, ref_scenes

SCENE_NAMES = {k: f.__name__ for k, f in ref_scenes.BY_SCENEID.items()}


def parse(argv=None):
    ap = argparse.ArgumentParser(prog="python -m srr.render_main", description=__doc__.split("\n\n")[0])
    ap.add_argument("--sceneid", type=int, default=2, choices=sorted(ref_scenes.BY_SCENEID),
                    help="; ".join(f"{k}: {v}" for k, v in SCENE_NAMES.items()))
    ap.add_argument("--nx", type=int, default=1000)
    ap.add_argument("--ny", type=int, default=1000)
    ap.add_argument("--ns", type=int, default=50, help="samples per pixel")
    ap.add_argument("--max-depth", type=int, default=50)
    ap.add_argument("--device", type=int, default=0)
    ap.add_argument("--gpus", type=int, default=1,
                    help="render on devices device .. device+gpus-1 (pixels dealt round-robin, one RCCL gather)")
    ap.add_argument("--contents", default=None, help="the reference's contents/ directory (assets)")
    ap.add_argument("--out", default="out.ppm")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    a = parse(argv)
    sc = ref_scenes.BY_SCENEID[a.sceneid](float(a.nx) / float(a.ny), contents=a.contents)  # :894-919
    r = (capi.Renderer(sc.text(), device=a.device) if a.gpus == 1 else
         capi.Renderer(sc.text(), devices=list(range(a.device, a.device + a.gpus))))
    t0 = time.perf_counter()
    out = r.render(a.nx, a.ny, a.ns, a.max_depth, tile=1)
    ms = (time.perf_counter() - t0) * 1e3
    print(f"{int(ms)}ms")  # :944-947
    capi.write_ppm(a.out, a.nx, a.ny, out["img8"])
    st = out["stats"]
    print(f"{SCENE_NAMES[a.sceneid]}: {a.nx}x{a.ny}x{a.ns}, {st['world_rays']} world rays, "
          f"{st['world_rays'] / max(ms, 1e-3) / 1e3:.1f} Msamples/s -> {a.out}", file=sys.stderr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
