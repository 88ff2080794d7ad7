"""Reduce tools/counters.sh's rocprofv3 passes to one JSON summary per kernel.

usage: python tools/counters.py PREFIX KERNEL_SUBSTR

Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES / SQ_BUSY_CYCLES / SQ_ACTIVE_* /
SQ_WAIT_* count quad-cycles; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~=
WAVE_CYCLES.  GRBM_GUI_ACTIVE is summed over the 8 XCDs.  FETCH_SIZE is KiB
and tallies 64 B per 128-B request on gfx950 (doubled); WRITE_SIZE is KiB.
"""
import collections
import csv
import glob
import hashlib
import json
import os
import sys

N_CU = 256


def main():
    prefix, kname = sys.argv[1], sys.argv[2]
    ctr = collections.defaultdict(list)
    dur = []
    for d in sorted(glob.glob(prefix + ".p*")):
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if kname in r["Kernel_Name"]:
                    ctr[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if kname in r["Kernel_Name"]:
                    dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    c = {k: sum(v) / len(v) for k, v in ctr.items()}  # per launch
    ms = 1e3 * sum(dur) / max(len(dur), 1)
    out = {"kernel": kname, "launches_profiled": len(dur), "ms_per_launch_profiled": round(ms, 3),
           "raw_per_launch": {k: v for k, v in sorted(c.items())}}
    g = lambda k: c.get(k, 0.0)
    if g("GRBM_GUI_ACTIVE") and ms:
        out["clock_ghz"] = round(g("GRBM_GUI_ACTIVE") / 8 / (ms * 1e-3) / 1e9, 3)
    if g("SQ_WAVE_CYCLES") and g("GRBM_GUI_ACTIVE"):
        cycles = g("GRBM_GUI_ACTIVE") / 8
        # resident waves per CU, time-averaged over the launch (quad-cycles x4)
        out["waves_per_cu_avg"] = round(4 * g("SQ_WAVE_CYCLES") / (N_CU * cycles), 2)
        out["waves_per_simd_avg"] = round(out["waves_per_cu_avg"] / 4, 2)
    if g("SQ_WAVE_CYCLES"):
        w = g("SQ_WAVE_CYCLES")
        out["wave_time_split"] = {"issuing": round(g("SQ_ACTIVE_INST_ANY") / w, 3),
                                  "waiting_on_memory_or_barrier": round(g("SQ_WAIT_ANY") / w, 3),
                                  "issue_stalled": round(g("SQ_WAIT_INST_ANY") / w, 3)}
    if g("SQ_ACTIVE_INST_VALU"):
        # lanes doing VALU work per VALU instruction (divergence), out of 64
        out["valu_lane_utilisation"] = round(g("SQ_THREAD_CYCLES_VALU") / (64 * g("SQ_ACTIVE_INST_VALU")), 3)
    if g("SQ_INSTS_VALU") and g("SQ_WAVES"):
        out["valu_insts_per_wave"] = round(g("SQ_INSTS_VALU") / g("SQ_WAVES"))
    if g("SQ_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
        out["sq_busy_frac"] = round(g("SQ_BUSY_CYCLES") * 4 / (g("GRBM_GUI_ACTIVE")), 3)
    if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
        rd, wr = g("FETCH_SIZE") * 1024 * 2, g("WRITE_SIZE") * 1024
        out["hbm"] = {"read_bytes": round(rd), "write_bytes": round(wr), "total_bytes": round(rd + wr),
                      "GBps_at_profiled_time": round((rd + wr) / (ms * 1e-3) / 1e9, 1) if ms else None}
    # the profiled frame (bench.py's JSON line of the first pass): bench.py prices
    # these per-launch counts per world ray on whatever frame it runs
    for log in sorted(glob.glob(prefix + ".p*.log")):
        lines = [l for l in open(log, errors="replace") if l.startswith("{")]
        if lines:
            b = json.loads(lines[-1])
            launches = b["roofline"].get("trace_launches") or 1
            out["world_rays_per_launch"] = round(b["config"]["world_rays_per_step"] * b["steps"] / launches)
            out["profiled_workload"] = b["config"]["workload"]
            break
    # the build these counters describe: bench.py prices a summary only on the same library
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.environ.get("SRR_LIB") or os.path.join(root, "simple-raytracing-render_amd", "libsrr.so")
    out["build"] = {"lib": os.path.relpath(lib, root), "lib_sha256": lib_sha256(lib),
                    "env": {k: v for k, v in sorted(os.environ.items()) if k.startswith("SRR_")}}
    print(json.dumps(out, indent=1))


def lib_sha256(path):
    """first 16 hex digits of the library's SHA-256 (bench.py compares them)"""
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


if __name__ == "__main__":
    main()
