"""Multi-device rendering through the C-ABI (srr_renderer_create_multi, SURVEY
§8(b).2-3, §8(e)): one process drives N GPUs -- the node-scale replacement for
the reference's 8 renderthreads in one process (Raytracing_n.cpp:932-941) --
and gathers the shards' slabs to device 0 over RCCL at frame end.

CPU tests: the shard / assembly bookkeeping (srr_multi_plan) for N = 1..8, and
the loud failure without a GPU.  GPU tests: the frame bitwise the one-device
frame with a real RCCL communicator at N = 1 (the leased box has one GPU) and
with N = 2..3 shards rehearsed on that one GPU (the gather then copies)."""
import os

import numpy as np
import pytest
import torch  # noqa: F401  (before libsrr's first HIP call: torch then brings its own HIP runtime)

from srr import capi, scenes


@pytest.mark.parametrize("nx,ny,tile", [(64, 48, 1), (37, 23, 4), (512, 512, 1), (1920, 1080, 16), (5, 3, 32)])
@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8])
def test_multi_plan_covers_the_frame_once(nx, ny, tile, n):
    """The packed frame holds every pixel exactly once; shard k's slab is the
    pixel list srr_shard_pixels deals shard k of n (the torch path's shards,
    srr/dist.py); scattering the packed slabs rebuilds the image."""
    p = capi.make_params(nx, ny, 4, 50, shard=(0, 1), tile=tile)
    index, off = capi.multi_plan(p, n)
    assert index.size == nx * ny and off[0] == 0 and off[-1] == nx * ny
    assert np.array_equal(np.sort(index), np.arange(nx * ny))
    for k in range(n):
        pk = capi.make_params(nx, ny, 4, 50, shard=(k, n), tile=tile)
        np.testing.assert_array_equal(index[off[k]:off[k + 1]], capi.shard_pixels(pk))
    img = np.random.default_rng(n).random((nx * ny, 3), dtype=np.float32)
    packed = np.concatenate([img[index[off[k]:off[k + 1]]] for k in range(n)])
    out = np.zeros_like(img)
    out[index] = packed  # k_scatter_pixels
    np.testing.assert_array_equal(out, img)
    if n > 1 and nx * ny >= 64 * n:  # balanced deal: shards within one tile row of each other
        sizes = np.diff(off)
        assert sizes.max() - sizes.min() <= tile * max(nx, ny)


def test_multi_plan_refuses_an_outer_shard():
    p = capi.make_params(64, 64, 4, 50, shard=(1, 2))
    with pytest.raises(capi.SrrError, match="shards the frame itself"):
        capi.multi_plan(p, 2)


def test_multi_renderer_fails_loudly_without_a_gpu():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is visible")
    sc, _ = scenes.s1_cornell()
    with pytest.raises(capi.SrrError, match="no HIP device"):
        capi.Renderer(sc.text(), devices=[0, 1])


def _frame(r, nx, ny, spp, tile, async_frames=0):
    import torch
    p = capi.make_params(nx, ny, spp, 50, tile=tile)
    if not async_frames:
        buf = torch.zeros((nx * ny, 3), dtype=torch.float32, device="cuda")
        st = r.render_device(p, buf.data_ptr())
        return [buf.cpu().numpy()], [st]
    bufs = [torch.zeros((nx * ny, 3), dtype=torch.float32, device="cuda") for _ in range(async_frames)]
    tickets = [r.render_device_async(p, b.data_ptr()) for b in bufs]
    sts = [r.wait(t) for t in tickets]
    return [b.cpu().numpy() for b in bufs], sts


@pytest.mark.gpu
def test_multi_rccl_one_device_is_bitwise_the_single_renderer():
    """A real RCCL communicator (ncclCommInitAll over the one leased GPU): the
    shard goes through ncclSend / ncclRecv to device 0 and k_scatter_pixels;
    the frame is bitwise srr_render's, world rays equal."""
    sc, _ = scenes.s2_cornell_teapot()
    text = sc.text()
    nx, ny, spp = 96, 80, 16
    one = capi.Renderer(text, device=0)
    want, wst = _frame(one, nx, ny, spp, 1)
    m = capi.Renderer(text, devices=[0])
    assert m.transport == "rccl" and m.devices() == [0]
    got, st = _frame(m, nx, ny, spp, 1)
    np.testing.assert_array_equal(got[0].view(np.uint32), want[0].view(np.uint32))
    assert st[0]["world_rays"] == wst[0]["world_rays"]
    # host entry point (srr_render: mean + tone map) through the same path
    h = m.render(nx, ny, spp)
    np.testing.assert_array_equal(h["mean"].view(np.uint32), want[0].view(np.uint32))
    # frames in flight (srr_render_device_async / wait): each bitwise the same
    frames, sts = _frame(m, nx, ny, spp, 1, async_frames=3)
    for f, s in zip(frames, sts):
        np.testing.assert_array_equal(f.view(np.uint32), want[0].view(np.uint32))
        assert s["world_rays"] == wst[0]["world_rays"]


@pytest.mark.gpu
@pytest.mark.parametrize("n,tile", [(2, 1), (3, 8)])
def test_multi_shards_rehearsed_on_one_gpu_are_bitwise_the_single_frame(n, tile):
    """n shards on the one leased GPU (device 0 repeated: the gather copies): the
    assembled frame is bitwise the one-device frame for the pixel deal of n GPUs,
    synchronous (one host thread per device) and pipelined."""
    sc, _ = scenes.s2_cornell_teapot()
    text = sc.text()
    nx, ny, spp = 72, 56, 8
    want, wst = _frame(capi.Renderer(text, device=0), nx, ny, spp, tile)
    m = capi.Renderer(text, devices=[0] * n)
    assert m.transport == "copy" and m.devices() == [0] * n
    got, st = _frame(m, nx, ny, spp, tile)
    np.testing.assert_array_equal(got[0].view(np.uint32), want[0].view(np.uint32))
    assert st[0]["world_rays"] == wst[0]["world_rays"]
    frames, sts = _frame(m, nx, ny, spp, tile, async_frames=2)
    for f in frames:
        np.testing.assert_array_equal(f.view(np.uint32), want[0].view(np.uint32))


@pytest.mark.gpu
def test_multi_refuses_kept_paths_and_forced_rccl_on_a_repeated_device(monkeypatch):
    sc, _ = scenes.s1_cornell()
    m = capi.Renderer(sc.text(), devices=[0, 0])
    with pytest.raises(capi.SrrError, match="fresh frames"):
        m.render(16, 16, 4, keep_paths=True)
    monkeypatch.setenv("SRR_MULTI_TRANSPORT", "rccl")
    with pytest.raises(capi.SrrError, match="distinct devices"):
        capi.Renderer(sc.text(), devices=[0, 0])
    assert os.environ["SRR_MULTI_TRANSPORT"] == "rccl"


@pytest.mark.gpu
def test_multi_fewer_pixels_than_devices_orders_the_scatter_after_the_callers_fill():
    """A frame with fewer pixels than shards (the last shard empty): the gather
    and scatter into the caller's image run after the caller's own work on it --
    here a fill of the image queued on the legacy stream right before the async
    render -- because device 0's exchange stream waits on that stream, not on any
    shard's frame: the image is the frame, not the fill."""
    import torch
    sc, _ = scenes.s1_cornell()
    text = sc.text()
    nx, ny, spp = 2, 1, 4
    want, _ = _frame(capi.Renderer(text, device=0), nx, ny, spp, 1)
    m = capi.Renderer(text, devices=[0, 0, 0])
    p = capi.make_params(nx, ny, spp, 50, tile=1)
    for _ in range(3):
        buf = torch.empty((nx * ny, 3), dtype=torch.float32, device="cuda")
        buf.fill_(7.0)
        t = m.render_device_async(p, buf.data_ptr())
        m.wait(t)
        np.testing.assert_array_equal(buf.cpu().numpy().view(np.uint32), want[0].view(np.uint32))


@pytest.mark.gpu
def test_multi_failed_index_allocation_leaves_no_stale_plan(monkeypatch):
    """The gather's pixel index is reallocated when a larger frame arrives; if that
    allocation fails (SRR_MULTI_FAIL_INDEX test hook), the renderer must not keep
    the old plan's key with a freed index: rendering the old size again restages
    and is bitwise the one-device frame."""
    sc, _ = scenes.s1_cornell()
    text = sc.text()
    m = capi.Renderer(text, devices=[0, 0])
    small, big = (24, 16), (40, 32)
    want, _ = _frame(capi.Renderer(text, device=0), *small, 4, 1)
    got, _ = _frame(m, *small, 4, 1)
    np.testing.assert_array_equal(got[0].view(np.uint32), want[0].view(np.uint32))
    monkeypatch.setenv("SRR_MULTI_FAIL_INDEX", "1")
    with pytest.raises(capi.SrrError, match="SRR_MULTI_FAIL_INDEX"):
        _frame(m, *big, 4, 1)
    monkeypatch.delenv("SRR_MULTI_FAIL_INDEX")
    got, _ = _frame(m, *small, 4, 1)
    np.testing.assert_array_equal(got[0].view(np.uint32), want[0].view(np.uint32))
    wbig, _ = _frame(capi.Renderer(text, device=0), *big, 4, 1)
    got, _ = _frame(m, *big, 4, 1)
    np.testing.assert_array_equal(got[0].view(np.uint32), wbig[0].view(np.uint32))
