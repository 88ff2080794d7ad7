"""Diagnostics: does torch's HIP initialisation still find the GPU after libsrr has run
work in the same process?  (tests/test_gpu_async.py failed with "No HIP GPUs are
available" whenever a test of tests/test_gpu_fullframe.py had rendered first in the same
pytest process; alone it passes.)  Run on the GPU box:

    python tools/torch_after_render.py STEP     STEP: create | render | render_keep

prints one JSON line: the step, torch.cuda.device_count(), and whether a torch tensor could be
made on the device afterwards (with the error text when not).  Round 6 found every step failing
while libsrr.so was loaded before torch (the process then runs /opt/rocm's HIP runtime, not
torch's); srr.capi now imports torch first, and every step passes."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "simple-raytracing-render_amd"))
from srr import capi, scenes  # noqa: E402


def main():
    step = sys.argv[1]
    sc, _ = scenes.s2_cornell_teapot()
    r = capi.Renderer(sc.text())
    if step == "render":
        r.render(64, 64, 4, 50)
    elif step == "render_keep":
        r.render(64, 64, 4, 50, keep_paths=True)
    out = {"step": step}
    import torch
    try:
        out["device_count"] = torch.cuda.device_count()
        t = torch.zeros(4, device="cuda")
        out["tensor_ok"] = bool(t.sum().item() == 0)
    except Exception as e:  # noqa: BLE001 -- the point is to report it
        out["tensor_ok"] = False
        out["error"] = str(e)[:200]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
