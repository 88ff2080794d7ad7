"""Reference vs restatement CPU rates on one pixel subset of the C2 frame,
single- and multi-core (SURVEY §8(d) calibration): the reference's own code
(oracle/_ref/ref_harness `sums`, one single-threaded process per core) and the
restatement (oracle/liboracle.so, its own thread pool), same pixels, same spp.

    python tools/cpu_calibration.py OUT.json [step] [cores]
"""
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracing-render_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import oracle_bind as ob  # noqa: E402
from srr import scenes  # noqa: E402


def ref_rate(scene, nx, ny, spp, step, procs):
    h = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    npix = nx * ny
    t0 = time.perf_counter()
    ps = [subprocess.Popen([h, "sums", scene, str(nx), str(ny), str(spp), "50", str(k * step), str(npix), "-",
                            str(procs * step)], stdout=subprocess.PIPE, text=True, cwd=os.path.dirname(scene))
          for k in range(procs)]
    outs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in ps]
    dt = time.perf_counter() - t0
    rays = sum(o["world_rays"] for o in outs)
    return {"msamples_per_s": rays / dt / 1e6, "world_rays": rays, "seconds": dt, "cores": procs}


def port_rate(text, nx, ny, spp, step, threads):
    pix = np.arange(0, nx * ny, step, dtype=np.int32)
    t0 = time.perf_counter()
    r = ob.render(text, nx, ny, spp, 50, pixels=pix, threads=threads, want_paths=False)
    dt = time.perf_counter() - t0
    rays = int(r["stats"][0])
    return {"msamples_per_s": rays / dt / 1e6, "world_rays": rays, "seconds": dt, "cores": threads}


def main():
    out = sys.argv[1]
    step = int(sys.argv[2]) if len(sys.argv) > 2 else 97
    cores = int(sys.argv[3]) if len(sys.argv) > 3 else (os.cpu_count() or 1)
    sc, _ = scenes.s2_cornell_teapot()
    text = sc.text()
    nx, ny, spp = 512, 512, 1024
    res = {"config": "C2 s2 512x512x1024, maxDepth 50", "pixels": f"every {step}th pixel ({len(range(0, nx * ny, step))})",
           "host": os.uname().nodename, "cpu_count": os.cpu_count()}
    with tempfile.TemporaryDirectory() as td:
        scene = os.path.join(td, "s.txt")
        open(scene, "w").write(text)
        ref_rate(scene, nx, ny, spp, step * 8, cores)  # warm-up: a cold first burst of processes runs slow
        res["reference_1"] = ref_rate(scene, nx, ny, spp, step, 1)
        res[f"reference_{cores}"] = ref_rate(scene, nx, ny, spp, step, cores)
    res["port_1"] = port_rate(text, nx, ny, spp, step, 1)
    res[f"port_{cores}"] = port_rate(text, nx, ny, spp, step, cores)
    for k in (1, cores):
        res[f"reference_over_port_{k}"] = res[f"reference_{k}"]["msamples_per_s"] / res[f"port_{k}"]["msamples_per_s"]
    assert res["reference_1"]["world_rays"] == res["port_1"]["world_rays"], "reference and restatement disagree"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
