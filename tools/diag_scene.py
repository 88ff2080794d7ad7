"""GPU vs CPU-restatement diagnostics for one reference builder on stand-in
assets: per-path error statistics, ray-count divergence, per-material split."""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "simple-raytracing-render_amd"), os.path.join(ROOT, "tests")]
import oracle_bind as ob  # noqa: E402
import parity  # noqa: E402
from srr import capi, ref_scenes  # noqa: E402
from test_ref_scenes import make_standin_contents  # noqa: E402

name = sys.argv[1]
nx, ny, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (24, 18, 4)
md = int(sys.argv[5]) if len(sys.argv) > 5 else 50
flags = int(sys.argv[6]) if len(sys.argv) > 6 else 0
root = make_standin_contents(tempfile.mkdtemp())
text = ref_scenes.BUILDERS[name](nx / ny, root).text()
out = capi.Renderer(text, device=0).render(nx, ny, spp, md, keep_paths=True, flags=flags)
ref = ob.render(text, nx, ny, spp, md)
g = out["paths"].reshape(-1, 3).astype(np.float64)
w = ref["paths"].reshape(-1, 3).astype(np.float64)
gr = out["rays"].reshape(-1).astype(int)
wr = ref["rays"].reshape(-1).astype(int)
pc = parity.compare_paths(out["paths"], ref["paths"])
print(name, "max_depth", md, "flags", flags, pc)
bad = np.array(pc["worst"] if False else np.flatnonzero(~np.isclose(g, w, rtol=1e-3, atol=1e-6, equal_nan=True).all(1)))
print("mismatching paths", len(bad), "of", len(g), "; of those with different ray counts:", int((gr[bad] != wr[bad]).sum()))
print("ray totals gpu/cpu", gr.sum(), wr.sum())
for i in bad[:int(os.environ.get("DIAG_N", "25"))]:
    print(i, "pix", i // spp, "s", i % spp, "rays", gr[i], wr[i], "gpu", g[i], "cpu", w[i])
