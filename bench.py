"""Benchmark: Msamples/s of the srr HIP path tracer on BASELINE.json's config
(Cornell box + Utah teapot, 6,400 triangles, 512x512, 1024 spp, MI355X).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

One step = one whole frame through the C-ABI (srr_render_device, inputs
resident in HBM) on every rank, then the frame-end exchange over RCCL
(srr/dist.py).  Default plan "tiles" (strong scaling, the
north_star split): the BASELINE config's one 512x512x1024 frame, tiles of edge
--tile (default 1: single pixels) dealt round-robin over the N GPUs (each tile row
rotated by one), one gather of the tiles' means to rank 0 (the image is bitwise
the 1-GPU image).  Plan "samples" (weak scaling): each GPU
renders 512x512x1024 paths as its sample range of one N*1024-spp frame; one
reduce of raw per-pixel sums.  A "sample" is one world ray segment (one
reference world->hit call).  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "simple-raytracing-render_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scene", default="s2",
                    choices=["s1", "s2", "s3", "s3_metal", "s4", "s5", "s4_real", "ball", "random"],
                    help="s4_real: the reference's real soldier_scene (Soilder.FBX, sky4.jpg; Raytracing_n.cpp:585-657) "
                         "from its committed fixture (tests/golden/make_soldier.py), 1920x1080x1024; ball: the "
                         "reference's as-shipped default run, sceneid 2 ball_scenes at its globals 1000x1000x50 "
                         "(Raytracing_n.cpp:39-43, :379-425); random: random_scene (~490 spheres, the global-memory "
                         "world variant of k_paths) at the same globals")
    ap.add_argument("--divs", type=int, default=0,
                    help="teapot subdivision (s2/s3: 10 = 6,400 tris; 100 = the reference's as-shipped 640,000, "
                         "teapot.h:77; s4/s5: 40 = 102,400)")
    ap.add_argument("--nx", type=int, default=0)
    ap.add_argument("--ny", type=int, default=0)
    ap.add_argument("--spp", type=int, default=0)
    ap.add_argument("--batch-paths", type=int, default=0)
    ap.add_argument("--tile", type=int, default=1,
                    help="tile edge of the tiles plan.  1 (pixels dealt round-robin, each row rotated by one) "
                         "balances the shards' COST, not just their rays: 8 C2 shards within 0.5 %% of their "
                         "mean time vs 10 %% at 16x16 and 12 %% at 32x32 (tools/shard_balance.py, "
                         "profiles/r03/shard_balance_*.json); a wave renders samples of one pixel, so smaller "
                         "tiles cost no coherence")
    ap.add_argument("--plan", default="tiles", choices=["tiles", "samples"],
                    help="multi-GPU split: tiles = strong scaling, the north_star split (one frame, --tile tiles "
                         "round-robin, one gather to rank 0; bitwise the 1-GPU image), samples = weak scaling "
                         "(each GPU renders spp samples of every pixel, one reduce of raw sums)")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="one frame at a time (srr_render_device) instead of two in flight "
                         "(srr_render_device_async: frame k+1's persistent blocks start on the CUs frame k's last "
                         "paths free, and frame k's exchange runs while frame k+1 renders)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--count-visits", action="store_true", help="diagnostic: count mesh box/triangle tests (slower)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--force-dist", action="store_true",
                    help="take the multi-rank code path even at world size 1 (init_process_group over "
                         "SRR_DIST_BACKEND, the frame-end gather/reduce through the collective): run under "
                         "torch.distributed.run --nproc-per-node 1 it executes the RCCL leg on one GPU")
    ap.add_argument("--host", default="torch", choices=["torch", "capi"],
                    help="torch: one process per GPU, the frame-end gather over torch.distributed (the driver's "
                         "torch.distributed.run launch); capi: ONE process drives --gpus N devices through the C-ABI "
                         "(srr_renderer_create_multi: a host thread or async frame per device, one RCCL "
                         "ncclSend/ncclRecv gather to device 0 from C++), run without torch.distributed.run")
    ap.add_argument("--rehearse", action="store_true",
                    help="--host capi on fewer GPUs than --gpus: the N shards share the visible devices (gather by "
                         "device copies instead of RCCL); for correctness rehearsals, not a scaling number")
    ap.add_argument("--save-frame", default="",
                    help="rank 0 saves the assembled frame of the last step (per-pixel means, .npy)")
    return ap.parse_args()


CONFIG_KEY = {"s1": "C1", "s2": "C2", "s3": "C3", "s3_metal": "C3_metal", "s4": "C4", "s5": "C5", "s4_real": "C4_real",
              "ball": "REF_ball_scenes", "random": "REF_random_scene"}


class _TextScene:
    def __init__(self, text):
        self._t = text

    def text(self):
        return self._t


def _soldier_real():
    import soldier_fixture
    return _TextScene(soldier_fixture.scene_text()), dict(nx=1920, ny=1080, spp=1024, max_depth=50)


def _ref_builder(name):
    """One of the reference's own scene builders (srr/ref_scenes.py, pinned to the
    reference's builder code) at the reference's globals nx = ny = 1000, ns = 50,
    maxDepth 50 (Raytracing_n.cpp:39-43), on its asset files (/root/reference/contents
    here, tests/golden/ref_assets.npz on the GPU box)."""
    from srr import ref_scenes
    contents = "/root/reference/contents"
    if not os.path.isdir(contents):
        import ref_fixtures
        contents = ref_fixtures.contents_dir()
    return ref_scenes.BUILDERS[name](1000 / 1000, contents), dict(nx=1000, ny=1000, spp=50, max_depth=50)


def host_cpus():
    """The host CPUs this process may run on: nproc (sched_getaffinity), capped by
    the cgroup CPU quota (cpu.max) when one is set -- on the GPU box the whole
    machine's CPUs are visible (os.cpu_count()) but a job's share is its quota."""
    nproc = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        pass
    return {"use": min(nproc, quota) if quota else nproc, "nproc": nproc, "cpu_count": os.cpu_count(),
            "cgroup_quota_cpus": quota}


def cpu_baseline(text, nx, ny, spp, budget_s):
    """The CPU restatement (oracle/liboracle.so, bit-identical to the
    reference) on a bounded pixel sample of the same frame."""
    import numpy as np

    import oracle_bind as ob
    threads = host_cpus()["use"]
    rng = np.random.default_rng(1)
    # calibrate on a small sample, then size the timed sample to ~budget_s
    n_cal = min(nx * ny, 4096)
    cal = np.sort(rng.choice(nx * ny, size=n_cal, replace=False)).astype(np.int32)
    t0 = time.perf_counter()
    r = ob.render(text, nx, ny, spp, 50, pixels=cal, threads=threads, want_paths=False)
    dt = max(time.perf_counter() - t0, 1e-3)
    n = int(min(nx * ny, max(n_cal, n_cal * budget_s / dt)))
    pix = np.sort(rng.choice(nx * ny, size=n, replace=False)).astype(np.int32)
    t0 = time.perf_counter()
    r = ob.render(text, nx, ny, spp, 50, pixels=pix, threads=threads, want_paths=False)
    dt = time.perf_counter() - t0
    rays = int(r["stats"][0])
    return {"value": rays / dt / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": f"{n} random pixels of the {nx}x{ny} frame x {spp} spp ({rays} world rays, {dt:.1f} s) "
                      f"on the CPU restatement oracle/restate.cpp (bit-exact to the reference)"}


def cpu_baseline_reference(text, nx, ny, spp, max_depth, budget_s):
    """The REFERENCE's own color() path (oracle/_ref/ref_harness, compiled from
    /root/reference's sources in the build container and shipped with the tree),
    deterministic per-path seeding, one single-threaded process per core over an
    evenly spaced pixel sample of the same frame (the whole frame when it fits
    the budget).  None when the harness binary is absent."""
    import subprocess
    import tempfile

    import numpy as np
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.access(harness, os.X_OK):
        return None
    cpus = host_cpus()
    procs = cpus["use"]
    npix = nx * ny
    with tempfile.TemporaryDirectory() as td:
        scene = os.path.join(td, "scene.txt")
        with open(scene, "w") as f:
            f.write(text)

        def run(p0, stride):
            return subprocess.Popen([harness, "sums", scene, str(nx), str(ny), str(spp), str(max_depth), str(p0),
                                     str(npix), "-", str(stride)], stdout=subprocess.PIPE, text=True,
                                    cwd=td)  # the reference opens its static outfile relative to the cwd (:45)

        # calibrate (and warm every core up: a cold first burst of processes runs
        # several times slower): each process ~32 pixels spread over the frame
        cstride = max(1, npix // (32 * procs))
        cal = [run((37 + k * cstride) % npix, procs * cstride) for k in range(procs)]
        cs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in cal]
        per_pix_s = max(max(c["ms"], 1e-3) * 1e-3 / max(c["pixels"], 1) for c in cs)
        step = max(1, int(np.ceil(npix * per_pix_s / (procs * budget_s))))  # every step-th pixel
        t0 = time.perf_counter()
        ps = [run(k * step, procs * step) for k in range(procs)]
        outs = [json.loads(p.communicate()[0].strip().splitlines()[-1]) for p in ps]
        dt = time.perf_counter() - t0
    rays = sum(o["world_rays"] for o in outs)
    pixels = sum(o["pixels"] for o in outs)
    what = "the whole frame" if step == 1 else f"every {step}th pixel ({pixels} pixels)"
    return {"value": rays / dt / 1e6, "unit": "Msamples/s", "cores": procs, "kind": "reference", "host_cpus": cpus,
            "sample": f"{what} of the {nx}x{ny} frame x {spp} spp ({rays} world rays, {dt:.1f} s): the "
                      f"reference's own color() (oracle/_ref/ref_harness, built from Raytracing_n.cpp), "
                      f"one single-threaded process per host CPU available to the job"}


def _lib_sha256(path):
    """first 16 hex digits of the library's SHA-256 (tools/counters.py records the same)"""
    import hashlib
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]
    except OSError:
        return None


def bench_line(a, text, cfg, nx, ny, spp, rays_total, elapsed, trace_ms, launches, world, workload_tail,
               parallelism, extra, rays_local=None, frame_spp=None, visits=None):
    """The JSON line (rank 0): value = every device's world rays over the slowest
    rank's time; the roofline prices rank 0's own rays (rays_local; all of them
    for --host capi, whose trace_ms / launches sum every device's) over its
    kernel time."""
    launches_total = launches
    rays = rays_total if rays_local is None else rays_local
    counts_json = json.load(open(os.path.join(ROOT, "tests", "golden", "traversal_counts.json")))
    key = CONFIG_KEY[a.scene]
    default_divs = {"s2": 10, "s3": 10, "s3_metal": 10, "s4": 40, "s5": 40}.get(a.scene)
    if a.divs and a.divs != default_divs:
        key = f"{key}_d{a.divs}"
    if key not in counts_json:
        raise SystemExit(f"no reference traversal counts for {key}: add it to tests/golden/make_counts.py")
    b_cfg = counts_json[key]["B_cfg"]
    value = rays_total / elapsed / 1e6
    # roofline of the dominant kernel (srr_trace) on rank 0: algorithmic bytes
    # (B_cfg per world ray, reference traversal counts) over its HIP-event time
    achieved = rays * b_cfg / (trace_ms * 1e-3) / 1e9 if trace_ms > 0 else None
    wave = bool(os.environ.get("SRR_ENGINE") == "wave")
    kernel_name = ("k_trace (wavefront engine)" if wave else
                   "k_paths (path-resident persistent kernel: trace + shade)")
    # measured HBM bytes: the counter summary of this build (below), else null
    traffic = None
    out = {
        "metric": "Msamples/s (rays x bounces) + HBM GB/s vs roofline, Cornell+teapot 1024spp",
        "value": round(value, 3),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak" if a.plan == "samples" else "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": ("the reference's own assets (Soilder.FBX mesh 0, sky4.jpg, textures) via the committed fixture"
                 if a.scene == "s4_real" else
                 "the reference's own scene builder and asset files (sky_2.png / sky_1 JPEGs)"
                 if a.scene in ("ball", "random") else
                 "synthetic (scene built in code: Cornell box + tessellated Utah teapot)"),
        "config": dict({"workload": f"{key}: {a.scene}{f' divs {a.divs}' if a.divs else ''} {nx}x{ny} {spp}spp "
                                    f"maxDepth {cfg['max_depth']}" + workload_tail,
                        "nx": nx, "ny": ny, "spp_per_gpu" if a.plan == "samples" else "spp": spp,
                        "frame_spp": frame_spp or spp, "world_rays_per_step": int(rays_total / a.steps),
                        "parallelism": parallelism}, **extra),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "kernel": kernel_name, "B_cfg": round(b_cfg, 1),
                     "trace_ms_per_launch": round(trace_ms / max(launches, 1), 4),
                     "trace_launches": launches_total,
                     "basis": "achieved/frac count ALGORITHMIC bytes: B_cfg per world ray from the "
                              "reference's traversal counts (SURVEY 8(d)); traffic is the measured HBM bytes",
                     "traffic_GBps": (round(traffic / (trace_ms / max(launches, 1) * 1e-3) / 1e9, 1)
                                      if traffic and trace_ms > 0 else None),
                     "measured_bound": "issue/latency: the scene lives in LDS and L2 (no counter summary of "
                                       "this config in profiles/)"},
    }
    # issue roofline of the same kernel from a committed PMC summary (tools/counters.sh ->
    # profiles/rNN/counters_<scene>.json, newest round first): VALU wave-instructions per
    # world ray of the profiled frame, times the world rays rank 0 traced here, over rank 0's
    # live kernel time -- so a shard, another frame size or another spp is priced by its own
    # rays, not by the profiled frame's -- against 1,024 SIMDs each issuing one wave64 VALU
    # instruction per 2 cycles (SIMD-32, MI355X_MICROARCH.md)
    cj, cnt = None, None
    suffix = key[len(CONFIG_KEY[a.scene]):]
    for rdir in sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]")), reverse=True):
        f = os.path.join(rdir, f"counters_{a.scene}{suffix}.json")
        if os.path.exists(f):
            j = json.load(open(f))
            if j.get("world_rays_per_launch"):
                cj, cnt = j, f
                break
    # a counter summary prices this run only when it profiled the library running here
    # (tools/counters.py records its SHA-256): instruction counts of another build are not
    # this kernel's
    from srr import capi
    sha = _lib_sha256(capi.LIB_PATH)
    out["roofline"]["build"] = {"lib": os.path.relpath(capi.LIB_PATH, ROOT), "lib_sha256": sha}
    if cj is not None and (cj.get("build") or {}).get("lib_sha256") != sha:
        out["roofline"]["issue"] = None
        out["roofline"]["issue_note"] = (
            f"{os.path.relpath(cnt, ROOT)} profiled library "
            f"{(cj.get('build') or {}).get('lib_sha256') or 'unrecorded'}, this run's is {sha}: its counters are "
            f"not this build's, so no issue roofline is derived from them")
        cj = None
    # a scene whose sphere runs go through sgroup_hit's BVH (ball_scenes, random_scene) does not
    # perform the reference's linear list of sphere tests that its B_cfg prices
    # (hitable_list.h:21-33): those bytes are not this kernel's traversal
    if a.scene in ("ball", "random") and not os.environ.get("SRR_SGROUP", "1") == "0":
        for k in ("achieved", "frac"):
            out["roofline"][k] = None
        out["roofline"]["frac_note"] = (
            f"B_cfg {b_cfg:.0f} B counts the reference's linear list ({counts_json[key].get('N_prim', '?')} "
            f"primitive tests per world ray); srr answers the list's sphere runs through a BVH (sgroup_hit) "
            f"with the same result, so the reference's algorithmic bytes would overstate this kernel's "
            f"traffic (frac > 1): not reported")
    if cj is not None and trace_ms > 0 and rays > 0:
        insts_per_ray = cj["raw_per_launch"]["SQ_INSTS_VALU"] / cj["world_rays_per_launch"]
        clock = cj.get("clock_ghz") or 2.4
        rate = insts_per_ray * rays / (trace_ms * 1e-3)
        peak = 1024 * clock * 1e9 / 2
        lane = cj.get("valu_lane_utilisation")
        out["roofline"]["issue"] = {
            "valu_wave_insts_per_s": round(rate, -6), "peak": round(peak, -6), "frac": round(rate / peak, 4),
            "lane_utilisation": lane, "lane_frac": round(rate / peak * lane, 4) if lane else None,
            "valu_wave_insts_per_world_ray": round(insts_per_ray, 3),
            "wave_time_split": cj.get("wave_time_split"), "clock_ghz": clock,
            "source": os.path.relpath(cnt, ROOT) + f" ({cj.get('ms_per_launch_profiled')} ms/launch profiled, "
                      f"{cj.get('profiled_workload', '?')})"}
        ws = cj.get("wave_time_split") or {}
        hbm = cj.get("hbm") or {}
        # the counter summary's HBM bytes (FETCH_SIZE / WRITE_SIZE passes of the same
        # profiling run) take precedence over an older separate traffic summary
        if hbm.get("total_bytes"):
            # measured HBM bytes per world ray of the profiled frame, priced on this run's launches
            traffic = round(hbm["total_bytes"] / cj["world_rays_per_launch"] * rays / max(launches, 1))
            out["roofline"]["traffic"] = traffic
            out["roofline"]["traffic_GBps"] = round(traffic / (trace_ms / max(launches, 1) * 1e-3) / 1e9, 1)
        out["roofline"]["measured_bound"] = (
            f"latency/issue: VALU pipe {100 * rate / peak:.0f}% busy at {100 * (lane or 0):.0f}% lane "
            f"utilisation, waves {100 * ws.get('waiting_on_memory_or_barrier', 0):.0f}% of their time waiting; "
            f"HBM {100 * (out['roofline']['traffic_GBps'] or 0) / HBM_PEAK_GBS:.1f}% of peak")
    if a.count_visits:
        out["visits"] = {"box_tests_per_ray": visits[0] / max(rays, 1), "tri_tests_per_ray": visits[1] / max(rays, 1),
                         "stack_overflows": visits[2], "note": "counting run: timing not representative"}
    if world == 1 and not a.no_cpu_baseline:
        # the reference's own code when its harness was built (oracle/_ref), else the
        # bit-exact restatement; the two are different harnesses (processes vs threads),
        # so neither calibrates the other
        ref = cpu_baseline_reference(text, nx, ny, spp, cfg["max_depth"], a.cpu_seconds)
        out["cpu_baseline"] = ref if ref is not None else cpu_baseline(text, nx, ny, spp, a.cpu_seconds)
    return out


def bench_capi(a, rend, devices, text, sc, cfg, nx, ny, spp, dev, n_dev):
    """--host capi: ONE process renders the whole frame over --gpus N devices
    through srr_renderer_create_multi (C++: a host thread / async frame per device,
    one RCCL gather of the shards' packed slabs to device 0, the scatter there).
    A step is one whole assembled frame; two frames in flight unless
    --no-pipeline."""
    import torch

    from srr import capi
    p = capi.make_params(nx, ny, spp, cfg["max_depth"], tile=a.tile, batch_paths=a.batch_paths,
                         flags=capi.FLAG_COUNT_VISITS if a.count_visits else 0)
    pipeline = not (a.no_pipeline or a.count_visits)
    bufs = [torch.zeros((nx * ny, 3), dtype=torch.float32, device=dev) for _ in range(2 if pipeline else 1)]

    def run_frames(n):
        if not pipeline:
            return [rend.render_device(p, bufs[0].data_ptr()) for _ in range(n)]
        stats, pend = [], []
        for k in range(n):
            pend.append(rend.render_device_async(p, bufs[k % 2].data_ptr()))
            if len(pend) == 2:
                stats.append(rend.wait(pend.pop(0)))
        stats += [rend.wait(t) for t in pend]
        return stats

    run_frames(a.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sts = run_frames(a.steps)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    rays = sum(st["world_rays"] for st in sts)
    trace_ms = sum(st["trace_ms"] for st in sts)
    launches = sum(st["trace_launches"] for st in sts)
    visits = [sum(st[k] for st in sts) for k in ("box_tests", "tri_tests", "stack_overflows")]
    if a.save_frame:
        import numpy as np
        np.save(a.save_frame, bufs[(a.steps - 1) % len(bufs)].cpu().numpy())
    out = bench_line(a, text, cfg, nx, ny, spp, rays, elapsed, trace_ms, launches, world=a.gpus,
                     workload_tail=(f", {a.tile}x{a.tile} tiles round-robin over {a.gpus} devices of ONE process "
                                    f"(srr_renderer_create_multi), one {rend.transport.upper()} gather to device 0"
                                    if a.gpus > 1 else f", whole frame on one GPU of ONE process "
                                    f"(srr_renderer_create_multi), one {rend.transport.upper()} gather to device 0"),
                     parallelism=f"tiles{a.gpus}", extra={"host": "capi", "devices": devices,
                                                          "transport": rend.transport, "devices_seen": n_dev,
                                                          "frames_in_flight": 2 if pipeline else 1},
                     visits=visits)
    print(json.dumps(out), flush=True)


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    from srr import capi, scenes
    from srr import dist as dist_frame

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # frame-end exchange backend: "nccl" (= RCCL over xGMI, one GPU per rank) or
    # "gloo" (host-staged gather; lets several ranks share one GPU, e.g. the
    # 2-rank rehearsal of tests/test_bench_multirank.py on a one-GPU box)
    backend = os.environ.get("SRR_DIST_BACKEND", "nccl")
    if a.host == "capi":
        if world != 1:
            raise SystemExit("--host capi is one process driving --gpus N devices: run it without torch.distributed.run")
        if a.plan != "tiles":
            raise SystemExit("--host capi renders the tiles plan (srr_renderer_create_multi)")
    if backend not in ("nccl", "gloo"):
        raise SystemExit(f"SRR_DIST_BACKEND must be nccl or gloo, not {backend!r}")
    n_dev = torch.cuda.device_count()  # counting devices does not initialise the GPU
    dev_idx = local % max(n_dev, 1)
    use_dist = (world > 1 or a.force_dist) and a.host == "torch"
    if a.force_dist and "MASTER_ADDR" not in os.environ:
        raise SystemExit("--force-dist: run under torch.distributed.run (MASTER_ADDR/MASTER_PORT unset)")
    dist_world = 1
    if use_dist:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group("gloo")
        dist_world = dist.get_world_size()
        if dist_world != world:
            raise SystemExit(f"communicator has {dist_world} ranks, WORLD_SIZE says {world}")
    if a.host == "capi":
        if n_dev < a.gpus and not a.rehearse:
            raise SystemExit(f"--host capi --gpus {a.gpus}: {n_dev} GPUs visible (--rehearse shares them)")
    elif a.gpus != world:
        raise SystemExit(f"--gpus {a.gpus} but {world} rank(s) were launched (use torch.distributed.run "
                         f"--nproc-per-node {a.gpus})")
    if backend == "nccl" and use_dist and n_dev < world:
        raise SystemExit(f"RCCL wants one GPU per rank: {world} ranks, {n_dev} GPUs visible")
    torch.cuda.set_device(dev_idx)
    dev = torch.device("cuda", dev_idx)
    host_reduce = use_dist and backend == "gloo"

    dv = {"divs": a.divs} if a.divs else {}
    if a.divs and a.scene in ("s1", "s4_real", "ball", "random"):
        raise SystemExit(f"--divs: {a.scene} has no teapot")
    fac = {"s1": scenes.s1_cornell, "s2": lambda: scenes.s2_cornell_teapot(**dv),
           "s3": lambda: scenes.s3_cornell_teapot_microfacet(**dv),
           "s3_metal": lambda: scenes.s3_cornell_teapot_microfacet("metal", **dv),
           "s4": lambda: scenes.s4_soldier_standin(**dv), "s5": lambda: scenes.s5_soldier_fog(**dv),
           "s4_real": _soldier_real, "ball": lambda: _ref_builder("ball_scenes"),
           "random": lambda: _ref_builder("random_scene")}[a.scene]
    sc, cfg = fac()
    nx, ny, spp = a.nx or cfg["nx"], a.ny or cfg["ny"], a.spp or cfg["spp"]
    text = sc.text()
    if a.host == "capi":
        devices = [k % max(n_dev, 1) for k in range(a.gpus)]
        rend = capi.Renderer(text, devices=devices)  # (at N = 1 too: an RCCL communicator of one device)
        return bench_capi(a, rend, devices, text, sc, cfg, nx, ny, spp, dev, n_dev)
    rend = capi.Renderer(text, device=dev_idx)
    sh = dist_frame.plan_shard(nx, ny, spp, cfg["max_depth"], rank, world, plan=a.plan, tile=a.tile,
                               batch_paths=a.batch_paths, flags=capi.FLAG_COUNT_VISITS if a.count_visits else 0)
    pipeline = not a.no_pipeline
    ex = dist_frame.FrameExchange(sh, dev, dist if use_dist else None, host_staged=host_reduce,
                                  buffers=2 if pipeline else 1)

    frame = [None]

    def run_frames(n):
        """n whole frames; returns their stats.  Pipelined: frame k is enqueued,
        then frame k-1 is waited for and exchanged (RCCL gather + assembly on rank
        0) from its own buffer while frame k renders."""
        stats = []
        if not pipeline:
            for _ in range(n):
                stats.append(rend.render_device(sh.params, ex.local.data_ptr()))
                frame[0] = ex.finish()  # frame-end exchange (RCCL gather) + assembly on rank 0
            return stats
        pend = []
        for k in range(n):
            buf = ex.locals[k % 2]
            pend.append((rend.render_device_async(sh.params, buf.data_ptr()), buf))
            if len(pend) == 2 or k == n - 1:
                while pend and (len(pend) == 2 or k == n - 1):
                    t, b = pend.pop(0)
                    stats.append(rend.wait(t))
                    frame[0] = ex.finish(b)
        return stats

    def barrier():
        if use_dist:
            dist.barrier()
        torch.cuda.synchronize()

    if a.count_visits:
        pipeline = False  # counted frames are synchronous (SRR_FLAG_COUNT_VISITS)
    run_frames(a.warmup)
    barrier()
    t0 = time.perf_counter()
    rays = 0
    trace_ms = 0.0
    launches = 0
    visits = [0, 0, 0]
    for st in run_frames(a.steps):
        visits = [visits[0] + st["box_tests"], visits[1] + st["tri_tests"], visits[2] + st["stack_overflows"]]
        rays += st["world_rays"]
        trace_ms += st["trace_ms"]
        launches += st["trace_launches"]
    barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed, float(rays), trace_ms], dtype=torch.float64,
                     device="cpu" if host_reduce else dev)
    if use_dist:
        tmax = t[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = t[1:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed = float(tmax.item())
        rays_total = float(tsum[0].item())
    else:
        rays_total = float(rays)
    if rank == 0 and a.save_frame:
        import numpy as np
        np.save(a.save_frame, frame[0].cpu().numpy())
    if rank == 0:
        coll = "RCCL" if backend == "nccl" else "host-staged gloo"
        tail = ((f", {a.tile}x{a.tile} tiles round-robin over {world} GPUs, one {coll} gather to rank 0 at frame end"
                 if use_dist else ", whole frame on one GPU (no collective)")
                if a.plan == "tiles" else
                f" per GPU; {world} GPU(s) render sample ranges of one {spp * world}spp frame" +
                (f", one {coll} reduce at frame end" if use_dist else ""))
        out = bench_line(a, text, cfg, nx, ny, spp, rays_total, elapsed, trace_ms, launches, world, tail,
                         f"{a.plan}{world}", {"host": "torch", "dist_backend": backend if use_dist else None,
                                              "dist_world": dist_world if use_dist else None, "devices_seen": n_dev,
                                              "frames_in_flight": 2 if pipeline else 1},
                         rays_local=rays, frame_spp=sh.total_spp, visits=visits)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
