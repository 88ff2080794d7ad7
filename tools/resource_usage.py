"""VGPRs / scratch / occupancy / LDS per kernel of csrc/kernels.hip.

usage: python tools/resource_usage.py [name-filter]   (compiles for gfx950, no GPU needed)
"""
import os
import re
import subprocess
import sys

PKG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "simple-raytracing-render_amd")
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-O3", "-fPIC", "-ffp-contract=off",
       "-mllvm", "-disable-machine-licm", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "-fno-slp-vectorize", "-fno-unroll-loops", *os.environ.get("EXTRA_HIPFLAGS", "").split(), "-c", "csrc/kernels.hip",
       "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, cwd=PKG, capture_output=True, text=True).stderr
flt = sys.argv[1] if len(sys.argv) > 1 else "k_paths"
cur, rows = None, {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
        cur = cur.replace("void srr::dev::", "").split("(")[0]
        rows[cur] = {}
        continue
    m = re.search(r"\s((?:VGPRs|SGPRs)(?: Spill)?|AGPRs|ScratchSize|Occupancy|LDS Size)[^:]*: (\d+)", line)
    if m and cur:
        rows[cur][m.group(1)] = int(m.group(2))
for k, v in rows.items():
    if flt in k:
        print(f"{k:45s} " + "  ".join(f"{a}={b}" for a, b in v.items()))
