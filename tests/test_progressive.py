"""Progressive rendering with resume (srr/progressive.py):
chunked sample ranges accumulate in sample order, so any chunking -- including
a save in one renderer and a resume in a fresh one -- is bitwise the one-shot
image; and the PPM writer reproduces the reference's own output files byte for
byte (Raytracing_n.cpp:873-886)."""
import glob
import os

import numpy as np
import pytest

from srr import capi, scenes
from srr.progressive import Progressive


def test_accum_symbols_exported():
    L = capi.lib()
    for name in ("srr_accum_get", "srr_accum_set", "srr_write_png", "srr_image_load", "srr_device_kat"):
        assert hasattr(L, name), name
    assert capi.FLAG_CONTINUE == 16


def _read_ppm(path):
    tok = open(path, "rb").read().split()
    assert tok[0] == b"P3"
    nx, ny, mx = int(tok[1]), int(tok[2]), int(tok[3])
    assert mx == 255
    return nx, ny, np.array([int(t) for t in tok[4:4 + 3 * nx * ny]], np.uint8).reshape(-1, 3)


@pytest.mark.parametrize("path", sorted(glob.glob("/root/reference/results/*.ppm"))[:2] or ["missing"])
def test_ppm_writer_matches_reference_outputs(path, tmp_path):
    if not os.path.exists(path):
        pytest.skip("reference results not present")
    nx, ny, px = _read_ppm(path)
    out = tmp_path / "o.ppm"
    capi.write_ppm(str(out), nx, ny, px)
    assert out.read_bytes() == open(path, "rb").read()


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, capi.FLAG_WAVEFRONT])
def test_progressive_chunks_equal_one_shot(flags, tmp_path):
    sc, _ = scenes.s3_cornell_teapot_microfacet()
    text = sc.text()
    nx, ny = 40, 30
    one = capi.Renderer(text).render(nx, ny, 12, 50, flags=flags)["mean"]
    r = capi.Renderer(text)
    pr = Progressive(r, nx, ny, 50, flags=flags)
    for n in (1, 4, 2):
        pr.step(n)
    state = str(tmp_path / "state.npz")
    pr.save(state)
    r2 = capi.Renderer(text)
    pr2 = Progressive(r2, nx, ny, 50, flags=flags)
    pr2.load(state)
    assert pr2.samples == 7
    pr2.step(5)
    np.testing.assert_array_equal(pr2.mean.view(np.uint32), one.view(np.uint32))
    pr.step(5)
    np.testing.assert_array_equal(pr.mean.view(np.uint32), one.view(np.uint32))


@pytest.mark.gpu
def test_continue_without_state_is_an_error():
    sc, _ = scenes.s1_cornell()
    r = capi.Renderer(sc.text())
    with pytest.raises(capi.SrrError):
        r.render(8, 8, 2, 50, flags=capi.FLAG_CONTINUE, sample_begin=2)


@pytest.mark.gpu
def test_continue_rejects_a_mismatched_resume():
    """The running sums know their sample count and their frame / shard: a
    resume at the wrong sample or with another shard is an error, and the sums
    survive it intact."""
    sc, _ = scenes.s1_cornell()
    r = capi.Renderer(sc.text())
    nx, ny = 32, 32
    r.render(nx, ny, 3, 50, shard=(0, 2), tile=16)
    with pytest.raises(capi.SrrError):  # 3 samples are in the sums, not 2
        r.render(nx, ny, 2, 50, shard=(0, 2), tile=16, flags=capi.FLAG_CONTINUE, sample_begin=2)
    with pytest.raises(capi.SrrError):  # same pixel count, other shard
        r.render(nx, ny, 2, 50, shard=(1, 2), tile=16, flags=capi.FLAG_CONTINUE, sample_begin=3)
    got = r.render(nx, ny, 2, 50, shard=(0, 2), tile=16, flags=capi.FLAG_CONTINUE, sample_begin=3)["mean"]
    want = capi.Renderer(sc.text()).render(nx, ny, 5, 50, shard=(0, 2), tile=16)["mean"]
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
