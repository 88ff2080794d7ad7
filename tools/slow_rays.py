"""Slow / NaN-bound world hits of one frame (diagnostics build, run via gpurun).

Build: make -C simple-raytracing-render_amd BUILD=build_slow OUT=libsrr_slow.so \\
         EXTRA_CXXFLAGS=-DSRR_SLOW_RAYS=100000 EXTRA_HIPFLAGS=-DSRR_SLOW_RAYS=100000
Run:   SRR_LIB=$PWD/simple-raytracing-render_amd/libsrr_slow.so python tools/slow_rays.py [--scene s2] [--shards N]

Every lane of a world hit slower than SRR_SLOW_RAYS ticks (100 MHz), and every
lane whose mesh walk took the NaN-bound scan (kernels.hip mesh_scan_nan), is
recorded by k_paths; this prints one JSON line per record with its pixel and
sample decoded (whole frame: identity pixel list), then a summary.
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def parse(lines):
    out = []
    for l in lines:
        if l.startswith("SLOWRAY "):
            s = re.sub(r"-?nan", "NaN", l.split("SLOWRAY ", 1)[1])
            out.append(json.loads(re.sub(r"(-?)inf\b", r"\1Infinity", s)))
    return out


def child(a):
    sys.path.insert(0, os.path.join(ROOT, "simple-raytracing-render_amd"))
    import torch
    from srr import capi, scenes
    from srr import dist as dist_frame
    sc, cfg = scenes.SCENES[a.scene]()
    nx, ny, spp = cfg["nx"], cfg["ny"], cfg["spp"]
    rend = capi.Renderer(sc.text(), device=0)
    sh = dist_frame.plan_shard(nx, ny, spp, cfg["max_depth"], a.shard, a.shards, plan="tiles", tile=a.tile)
    out = torch.zeros((len(sh.pixels), 3), dtype=torch.float32, device="cuda:0")
    st = rend.render_device(sh.params, out.data_ptr())
    print(json.dumps({"total_ms": st["total_ms"], "world_rays": st["world_rays"]}), file=sys.stderr, flush=True)
    import numpy as np
    np.save(a.pix_out, sh.pixels)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="s2")
    ap.add_argument("--shards", type=int, default=1)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--tile", type=int, default=16)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("--pix-out", default="/tmp/slow_pixels.npy")
    a = ap.parse_args()
    if a.child:
        return child(a)
    import numpy as np
    res = []
    for k in range(a.shards):
        p = subprocess.run([sys.executable, __file__, "--child", "--scene", a.scene, "--shards", str(a.shards),
                            "--shard", str(k), "--tile", str(a.tile), "--pix-out", a.pix_out],
                           capture_output=True, text=True, timeout=600)
        if p.returncode != 0:
            sys.exit(p.stderr[-2000:])
        recs = parse(p.stderr.splitlines())
        stats = [json.loads(l) for l in p.stderr.splitlines() if l.startswith('{"total_ms"')][-1]
        pix = np.load(a.pix_out)
        for r in recs:
            lp, s = divmod(r["g"], r["spp_w"])
            r["pixel"] = int(pix[lp])
            r["sample"] = s
            r["shard"] = k
            print(json.dumps(r))
        nan_lanes = [r for r in recs if (r["steps"] >> 28) & 1]
        slow = [r for r in recs if r["ticks"] > 100000]
        res.append({"shard": k, "of": a.shards, "total_ms": round(stats["total_ms"], 3), "records": len(recs),
                    "nan_bound_lanes": len(nan_lanes), "max_world_hit_ms": max((r["ticks"] for r in recs), default=0) * 1e-5,
                    "slow_lanes_over_1ms": len(slow)})
        print(json.dumps(res[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"summary": res}))


if __name__ == "__main__":
    main()
