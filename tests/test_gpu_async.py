"""srr_render_device_async / srr_render_wait (include/srr_capi.h): frames in
flight on the renderer's two frame slots are bitwise the frames of the
synchronous srr_render_device, whatever is enqueued or waited in between."""
import numpy as np
import pytest

from srr import capi, scenes

pytestmark = pytest.mark.gpu


def _setup(nx=48, ny=40, spp=16):
    import torch
    sc, _ = scenes.s2_cornell_teapot()
    r = capi.Renderer(sc.text())
    p = capi.make_params(nx, ny, spp, 50)
    bufs = [torch.zeros((nx * ny, 3), dtype=torch.float32, device="cuda") for _ in range(3)]
    return r, p, bufs


def _bits(t):
    return t.cpu().numpy().view(np.uint32)


def test_async_frames_equal_the_synchronous_frame():
    import torch
    r, p, bufs = _setup()
    st = r.render_device(p, bufs[0].data_ptr())
    torch.cuda.synchronize()
    want = _bits(bufs[0])
    t1 = r.render_device_async(p, bufs[1].data_ptr())
    t2 = r.render_device_async(p, bufs[2].data_ptr())
    s1, s2 = r.wait(t1), r.wait(t2)
    np.testing.assert_array_equal(_bits(bufs[1]), want)
    np.testing.assert_array_equal(_bits(bufs[2]), want)
    assert s1["world_rays"] == s2["world_rays"] == st["world_rays"]
    assert s1["paths"] == st["paths"] and s1["trace_launches"] == st["trace_launches"]


def test_third_frame_finishes_the_oldest_and_waits_out_of_order():
    import torch
    r, p, bufs = _setup(32, 24, 8)
    st = r.render_device(p, bufs[0].data_ptr())
    torch.cuda.synchronize()
    want = _bits(bufs[0])
    outs = [torch.zeros_like(bufs[0]) for _ in range(4)]
    tickets = [r.render_device_async(p, o.data_ptr()) for o in outs]  # 4 frames, 2 slots
    for t in reversed(tickets):  # any wait order
        assert r.wait(t)["world_rays"] == st["world_rays"]
    for o in outs:
        np.testing.assert_array_equal(_bits(o), want)
    with pytest.raises(capi.SrrError):
        r.wait(tickets[0])  # each ticket once


def test_async_with_synchronous_frames_and_shard_changes_in_between():
    import torch
    r, p, bufs = _setup(40, 32, 8)
    whole = torch.zeros_like(bufs[0])
    r.render_device(p, whole.data_ptr())
    torch.cuda.synchronize()
    whole_np = whole.cpu().numpy()
    t1 = r.render_device_async(p, bufs[1].data_ptr())
    # a tile shard of the same frame: a new pixel list while t1 is in flight
    ps = capi.make_params(40, 32, 8, 50, shard=(1, 3), tile=8)
    pix = capi.shard_pixels(ps)
    part = torch.zeros((pix.size, 3), dtype=torch.float32, device="cuda")
    t2 = r.render_device_async(ps, part.data_ptr())
    sync = torch.zeros_like(bufs[0])
    r.render_device(p, sync.data_ptr())  # synchronous frame while t2 may still run
    r.wait(t2)
    r.wait(t1)
    np.testing.assert_array_equal(bufs[1].cpu().numpy().view(np.uint32), whole_np.view(np.uint32))
    np.testing.assert_array_equal(sync.cpu().numpy().view(np.uint32), whole_np.view(np.uint32))
    np.testing.assert_array_equal(part.cpu().numpy().view(np.uint32), whole_np[pix].view(np.uint32))


def test_async_refuses_progressive_and_kept_paths():
    import torch
    r, p, bufs = _setup(16, 16, 4)
    for flags in (capi.FLAG_KEEP_PATHS, capi.FLAG_CONTINUE, capi.FLAG_WAVEFRONT, capi.FLAG_COUNT_VISITS):
        q = capi.make_params(16, 16, 4, 50, flags=flags)
        with pytest.raises(capi.SrrError):
            r.render_device_async(q, bufs[0].data_ptr())
    torch.cuda.synchronize()


def test_alternating_sync_and_async_frames_keep_their_windows():
    """Synchronous and pipelined frames interleaved frame by frame: each
    mode keeps its sample window across the switches, every frame bitwise the
    same."""
    import torch
    r, p, bufs = _setup(40, 24, 8)
    r.render_device(p, bufs[0].data_ptr())
    torch.cuda.synchronize()
    want = _bits(bufs[0])
    for k in range(3):
        t = r.render_device_async(p, bufs[1].data_ptr())
        r.render_device(p, bufs[2].data_ptr())
        r.wait(t)
        np.testing.assert_array_equal(_bits(bufs[1]), want)
        np.testing.assert_array_equal(_bits(bufs[2]), want)
