"""Tile-plan load balance measured on ONE GPU (run via gpurun from the repo root).

For N in 2, 4, 8 it renders each rank's shard of the bench frame (srr/dist.py
plan "tiles", srr_shard_pixels) in turn on cuda:0 and reports the per-shard
render time (srr_stats.total_ms, HIP events around the whole render): the
busiest shard bounds an N-GPU strong-scaling step, so
    predicted efficiency = T(whole frame) / (N * max_k T(shard k)).
This is not a multi-GPU measurement (no RCCL exchange, one card): it isolates
the split's balance and the per-launch fixed costs of smaller shards.

    python tools/shard_balance.py [--scene s2] [--reps 2] [--tile 32] > gpurun_out/shard_balance.json
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracing-render_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="s2", choices=["s2", "s4"])
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--tile", type=int, default=32)
    ap.add_argument("--pipeline", type=int, default=0,
                    help="time N frames of each shard with two in flight (srr_render_device_async, as bench.py) "
                         "by the host clock, instead of the best single synchronous render")
    a = ap.parse_args()
    import torch

    from srr import capi, scenes
    from srr import dist as dist_frame
    sc, cfg = {"s2": scenes.s2_cornell_teapot, "s4": scenes.s4_soldier_standin}[a.scene]()
    nx, ny, spp, md = cfg["nx"], cfg["ny"], cfg["spp"], cfg["max_depth"]
    rend = capi.Renderer(sc.text(), device=0)

    def time_shard(k, n):
        sh = dist_frame.plan_shard(nx, ny, spp, md, k, n, plan="tiles", tile=a.tile)
        out = torch.zeros((len(sh.pixels), 3), dtype=torch.float32, device="cuda:0")
        rend.render_device(sh.params, out.data_ptr())  # warm-up (pixel list, Sobol set)
        if a.pipeline:
            import time
            outs = [out, torch.zeros_like(out)]
            best = None
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                pend = []
                for f in range(a.pipeline):
                    pend.append(rend.render_device_async(sh.params, outs[f % 2].data_ptr()))
                    if len(pend) == 2:
                        rays = rend.wait(pend.pop(0))["world_rays"]
                for t in pend:
                    rays = rend.wait(t)["world_rays"]
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) * 1e3 / a.pipeline
                best = ms if best is None else min(best, ms)
            return best, rays
        best = None
        rays = 0
        for _ in range(a.reps):
            st = rend.render_device(sh.params, out.data_ptr())
            best = st["total_ms"] if best is None else min(best, st["total_ms"])
            rays = st["world_rays"]
        return best, rays

    t1, r1 = time_shard(0, 1)
    res = {"scene": a.scene, "tile": a.tile, "pipelined_frames": a.pipeline, "frame": f"{nx}x{ny}x{spp}", "whole_frame_ms": round(t1, 3), "world_rays": r1,
           "splits": []}
    for n in (2, 4, 8):
        ts, rs = zip(*(time_shard(k, n) for k in range(n)))
        assert sum(rs) == r1, (n, sum(rs), r1)
        res["splits"].append({"n": n, "shard_ms": [round(t, 3) for t in ts],
                              "max_over_mean_ms": round(max(ts) / (sum(ts) / n), 4),
                              "max_over_mean_rays": round(max(rs) / (sum(rs) / n), 4),
                              "predicted_efficiency": round(t1 / (n * max(ts)), 4)})
        print(json.dumps(res["splits"][-1]), file=sys.stderr, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
