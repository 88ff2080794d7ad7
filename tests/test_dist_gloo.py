"""World-size-2 rehearsal of the multi-GPU frame path (srr/dist.py)
on CPU with the gloo backend.  Each rank's "render" is the CPU restatement
(oracle) of exactly the shard the plan assigns it; the frame-end exchange and
assembly are the product code bench.py runs over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_bind as ob
from srr import dist as dist_frame
from srr import scenes

NX, NY, SPP = 40, 24, 4  # ragged tiles at tile=16 (40 = 2.5 tiles)


def _scene_text():
    sc, _ = scenes.s2_cornell_teapot(divs=4)
    return sc.text()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, plan, text, outdir, staged=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sh = dist_frame.plan_shard(NX, NY, SPP, 50, rank, world, plan=plan, tile=16)
        ex = dist_frame.FrameExchange(sh, torch.device("cpu"), dist, host_staged=staged)
        if plan == "tiles":
            r = ob.render(text, NX, NY, SPP, 50, pixels=sh.pixels, want_paths=False)
            ex.local[:sh.pixels.size] = torch.from_numpy(r["img"])
        else:
            full = ob.render(text, NX, NY, SPP * world, 50, want_paths=True)
            mine = np.nan_to_num(full["paths"][:, rank * SPP:(rank + 1) * SPP, :], nan=0.0)  # de_nan
            acc = np.zeros((NX * NY, 3), np.float32)
            for k in range(SPP):  # the renderer's raw running sums (SRR_FLAG_SUMS), in sample order
                acc += mine[:, k]
            ex.local[:] = torch.from_numpy(acc)
        img = ex.finish()
        if rank == 0:
            np.save(os.path.join(outdir, f"{plan}.npy"), img.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("plan,world,staged", [("tiles", 2, False), ("tiles", 3, False), ("tiles", 8, False),
                                               ("samples", 2, False), ("samples", 8, True),
                                               ("tiles", 2, True), ("samples", 2, True)])
def test_multi_rank_frame_matches_single_render(plan, world, staged, tmp_path):
    """tiles: the gathered frame is bitwise the one-renderer frame; samples: the
    reduced raw sums give the world*spp frame up to summation order.  staged:
    the host-staged exchange bench.py uses with SRR_DIST_BACKEND=gloo."""
    text = _scene_text()
    mp.spawn(_rank_main, args=(world, _free_port(), plan, text, str(tmp_path), staged), nprocs=world, join=True)
    img = np.load(tmp_path / f"{plan}.npy")
    if plan == "tiles":
        ref = ob.render(text, NX, NY, SPP, 50, want_paths=False)["img"]
        np.testing.assert_array_equal(img, ref)  # bitwise: each pixel rendered whole on one rank
    else:
        ref = ob.render(text, NX, NY, SPP * world, 50, want_paths=False)["img"]
        np.testing.assert_allclose(img, ref, rtol=1e-5, atol=1e-6)  # partial sums per rank


def test_plans_cover_frame_once():
    for world in (1, 2, 3, 8):
        cover = np.zeros(NX * NY, np.int32)
        for k in range(world):
            sh = dist_frame.plan_shard(NX, NY, SPP, 50, k, world, plan="tiles", tile=16)
            cover[sh.pixels] += 1
            assert sh.counts[k] == sh.pixels.size
        assert (cover == 1).all()
        begins = [dist_frame.plan_shard(NX, NY, SPP, 50, k, world, plan="samples").params.sample_begin
                  for k in range(world)]
        assert begins == [k * SPP for k in range(world)]


def test_sobol_prefix_stable():
    """Sample sharding relies on the Sobol set being a prefix-stable sequence."""
    from srr import capi
    a, b = capi.sobol_points(1024), capi.sobol_points(4096)
    np.testing.assert_array_equal(a, b[:1024])
