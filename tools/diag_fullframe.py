"""Bisect a full-frame mismatch saved by tests/test_gpu_fullframe.py
(SRR_DIAG_DIR/<name>_diff.npz): re-render the failing pixels with the CPU
restatement and list the differing paths (pixel, sample, rays, radiance).
    python tools/diag_fullframe.py gpurun_out/c2_full_diff.npz [c2_full]"""
import sys

import numpy as np

sys.path[:0] = ["simple-raytracing-render_amd", "tests"]
import fullframe  # noqa: E402
import oracle_bind as ob  # noqa: E402

z = np.load(sys.argv[1])
name = sys.argv[2] if len(sys.argv) > 2 else "c2_full"
m = fullframe.meta(name)
pix = z["pixels"].astype(np.int32)
ref = ob.render(fullframe.scene_text(name), m["nx"], m["ny"], m["spp"], m["max_depth"], pixels=pix, threads=8)
gp, rp = z["paths"], ref["paths"]
gr, rr = z["rays"], ref["rays"]
gb, rb = gp.view(np.uint32), rp.view(np.uint32)
nan = np.isnan(gp) & np.isnan(rp)
diff = ~(((gb == rb) | nan).all(axis=2)) | (gr != rr)
print("pixels", pix.size, "differing paths", int(diff.sum()), "ray delta", int(gr.sum(dtype=np.int64)) - int(rr.sum(dtype=np.int64)))
ks = np.argwhere(diff)
for k, s in ks[:40]:
    p = int(pix[k])
    print(f"pix {p} (i={p % m['nx']}, j={m['ny'] - 1 - p // m['nx']}) s={s} rays gpu {gr[k, s]} ref {rr[k, s]}  L gpu {gp[k, s]} ref {rp[k, s]}")
np.save("/tmp/ff_bad_paths.npy", np.array([(int(pix[k]), int(s)) for k, s in ks], dtype=np.int64))
