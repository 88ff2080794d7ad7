"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes to HBM bytes per launch
of one kernel, written as the JSON bench.py reads for roofline.traffic.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR OUT.json [BENCH_LOG]

BENCH_LOG (bench.py's output of the profiled run) adds the frame's world rays
per launch, so bench.py can price the bytes per world ray on any frame.

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE and
WRITE_SIZE are reported in KiB; on gfx950 FETCH_SIZE counts 64 B per 128-B
fabric read request, so it is doubled.  The doubling is calibrated for wide
coalesced reads; the trace kernel's node/triangle gathers are 16 B per lane,
so the absolute number carries that caveat (ratios between variants do not).
"""
import csv
import glob
import json
import sys


def per_launch(d, counter, kernel):
    vals = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {counter} rows for kernel '{kernel}' under {d}")
    return sum(vals) / len(vals), len(vals)


def main():
    fdir, wdir, kernel, out = sys.argv[1:5]
    fetch_kib, n_f = per_launch(fdir, "FETCH_SIZE", kernel)
    write_kib, n_w = per_launch(wdir, "WRITE_SIZE", kernel)
    read_b = fetch_kib * 1024.0 * 2.0
    write_b = write_kib * 1024.0
    res = {
        "kernel": kernel,
        "launches": {"fetch": n_f, "write": n_w},
        "fetch_size_kib_raw": round(fetch_kib, 3),
        "write_size_kib_raw": round(write_kib, 3),
        "read_bytes_per_launch": round(read_b),
        "write_bytes_per_launch": round(write_b),
        "hbm_bytes_per_launch": round(read_b + write_b),
        "corrections": "FETCH_SIZE KiB x1024 x2 (gfx950 64B-per-128B-request tally); WRITE_SIZE KiB x1024",
    }
    if len(sys.argv) > 5:
        lines = [l for l in open(sys.argv[5], errors="replace") if l.startswith("{")]
        b = json.loads(lines[-1])
        launches = b["roofline"].get("trace_launches") or 1
        res["world_rays_per_launch"] = round(b["config"]["world_rays_per_step"] * b["steps"] / launches)
        res["hbm_bytes_per_world_ray"] = round(res["hbm_bytes_per_launch"] / res["world_rays_per_launch"], 2)
        res["profiled_workload"] = b["config"]["workload"]
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
