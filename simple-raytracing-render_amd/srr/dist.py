"""Multi-GPU frame rendering: one process per GPU, torch.distributed over RCCL
(gloo on CPU for tests).  SURVEY.md §8(e).

Every (pixel, sample) path is independent and the scene is read-only, so a
frame shards with no exchange until the end.  Two plans:

* ``tiles``   (strong scaling, a fixed frame; the default): rank k renders the
  tiles t of edge ``tile`` (bench.py default 1: single pixels) in tile row tr
  with (t + tr) % world == k, all samples: round
  robin with each tile row rotated by one, so no rank gets whole tile columns
  (srr_shard_pixels).  Frame end: one gather of
  the packed per-pixel means to rank 0, which scatters them into the image.
  Bitwise equal to the one-GPU image (each pixel's samples are summed on one
  GPU in sample order).
* ``samples`` (weak scaling, fixed work per GPU): rank k renders every pixel
  with samples [k*spp, (k+1)*spp) of one frame of world*spp samples per pixel
  (the per-path seeds and Sobol points are the global sample index's, so
  rank 0's slice is exactly the one-GPU spp frame).  Each rank outputs its raw
  per-pixel sample sums (SRR_FLAG_SUMS); frame end: one reduce(sum) to rank 0,
  which takes the mean as the renderer does (sum * (1/ns)).  Equal to the
  one-GPU world*spp frame up to float summation order (partial sums per rank).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import capi

PLANS = ("tiles", "samples")


@dataclass
class Shard:
    rank: int
    world: int
    plan: str
    params: capi.Params          # what this rank renders
    pixels: np.ndarray           # PPM-order pixel indices this rank outputs (ascending)
    counts: list                 # pixels per rank (tiles) / frame pixels (samples)
    total_spp: int               # samples per pixel of the assembled frame


def plan_shard(nx, ny, spp, max_depth, rank, world, plan="tiles", tile=32, batch_paths=0, flags=0) -> Shard:
    """Split one frame over `world` ranks.  `spp` is the frame's samples per
    pixel for ``tiles`` and the per-rank samples per pixel for ``samples``."""
    if plan not in PLANS:
        raise ValueError(f"plan must be one of {PLANS}")
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    if plan == "tiles":
        p = capi.make_params(nx, ny, spp, max_depth, shard=(rank, world), tile=tile, batch_paths=batch_paths,
                             flags=flags)
        counts = [capi.shard_pixels(capi.make_params(nx, ny, spp, shard=(k, world), tile=tile)).size
                  for k in range(world)]
        return Shard(rank, world, plan, p, capi.shard_pixels(p), counts, spp)
    p = capi.make_params(nx, ny, spp, max_depth, shard=(0, 1), tile=tile, batch_paths=batch_paths,
                         flags=flags | capi.FLAG_SUMS, sample_begin=rank * spp)
    return Shard(rank, world, plan, p, np.arange(nx * ny, dtype=np.int32), [nx * ny] * world, spp * world)


def shard_pixels_of(sh: Shard, k: int) -> np.ndarray:
    """Pixel list of rank k under the same plan (rank 0 scatters with these)."""
    if sh.plan == "samples":
        return sh.pixels
    p = capi.make_params(sh.params.nx, sh.params.ny, sh.params.spp, shard=(k, sh.world), tile=sh.params.tile)
    return capi.shard_pixels(p)


class FrameExchange:
    """Frame-end exchange for one plan, with buffers allocated once.

    `local` is this rank's [n_max, 3] float32 tensor of per-pixel means
    (``tiles``; rows beyond its pixel count are ignored) or sample sums
    (``samples``).  `finish()` returns the assembled [nx*ny, 3] frame of means
    on rank 0 (None elsewhere).  With one rank and no communicator, in PPM
    order, that frame is a VIEW of the buffer it was rendered into: with
    buffers=2, the frame two steps later overwrites it (copy it to keep it).
    With a communicator (``dist``) the collective runs even at world size 1
    (bench.py --force-dist: the RCCL leg on one GPU).

    host_staged: the collective runs on host copies (gloo, which has no gather
    or reduce of device tensors), so several ranks may share one GPU; the
    assembled frame is the same bits as over RCCL."""

    def __init__(self, sh: Shard, device, dist=None, host_staged=False, buffers=1):
        import torch
        self.sh, self.dist, self.torch = sh, dist, torch
        self.host_staged = bool(host_staged and dist is not None)
        nx, ny = sh.params.nx, sh.params.ny
        self.n_max = max(sh.counts)
        # `buffers` local outputs: two let frame k+1 render (srr_render_device_async)
        # while frame k is exchanged from the other
        self.locals = [torch.zeros((self.n_max, 3), dtype=torch.float32, device=device) for _ in range(buffers)]
        self.local = self.locals[0]
        self.image = torch.zeros((nx * ny, 3), dtype=torch.float32, device=device)
        xdev = "cpu" if self.host_staged else device  # where the collective's buffers live
        self.xlocal = torch.zeros((self.n_max, 3), dtype=torch.float32, device=xdev) if self.host_staged else None
        if sh.plan == "tiles":
            self.gathered = ([torch.zeros((self.n_max, 3), dtype=torch.float32, device=xdev)
                              for _ in range(sh.world)] if sh.rank == 0 else None)
            pix = [shard_pixels_of(sh, k) for k in range(sh.world)]
            self.idx = [torch.from_numpy(p.astype(np.int64)).to(device) for p in pix]
            # one rank whose shard is the frame in PPM order: the local means ARE the frame
            self.identity = sh.world == 1 and np.array_equal(pix[0], np.arange(nx * ny))
        # the renderer's mean: sum * (float)(1.0 / (float)ns)  (kernels.hip k_finish)
        self.inv_ns = torch.tensor(np.float32(1.0 / float(np.float32(sh.total_spp))), device=device)

    def finish(self, local=None):
        sh, torch = self.sh, self.torch
        local = self.local if local is None else local
        if sh.plan == "tiles":
            if self.dist is None:
                if self.identity:
                    return local[:sh.counts[0]]  # (a view of the buffer the frame was rendered into)
                self.image[self.idx[0]] = local[:sh.counts[0]]
                return self.image
            if self.host_staged:
                self.xlocal.copy_(local)
                self.dist.gather(self.xlocal, self.gathered, dst=0)
            else:
                self.dist.gather(local, self.gathered, dst=0)  # one exchange over RCCL / xGMI
            if sh.rank != 0:
                return None
            for k in range(sh.world):
                self.image[self.idx[k]] = self.gathered[k][:sh.counts[k]].to(self.image.device)
            return self.image
        # samples: raw per-pixel sums of this rank's samples, reduced to rank 0
        if self.dist is not None:
            if self.host_staged:
                self.xlocal.copy_(local)
                self.dist.reduce(self.xlocal, dst=0)
                if sh.rank == 0:
                    local.copy_(self.xlocal)
            else:
                self.dist.reduce(local, dst=0)
            if sh.rank != 0:
                return None
        torch.mul(local, self.inv_ns, out=self.image)
        return self.image
