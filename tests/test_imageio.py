"""Image decoding for textures: srr's PNG / baseline-JPEG /
TGA / BMP decoder behind srr_image_load and srr_image_texture_file must return
exactly what the reference's stbi_load (stb_image v2.19, Raytracing_n.cpp:26-27)
returns.

* Pinned: every image file the reference ships, decoded by the reference's own
  stbi_load in oracle/ref's harness; digests in tests/golden/images.json
  (tests/golden/make_images.py).  Runs where /root/reference is present.
* Synthetic: PNG colour types / bit depths / filters / Adam7, TGA (raw, RLE,
  both origins), BMP (24-bit both row orders, 8-bit palette) built here with
  their expected pixels; the lossless formats have one correct answer.
"""
import ctypes
import hashlib
import json
import os
import struct
import zlib

import numpy as np
import pytest

from srr import capi

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
GOLD = json.load(open(os.path.join(HERE, "golden", "images.json")))


@pytest.mark.parametrize("key", sorted(GOLD))
def test_reference_images_match_stbi_load(key):
    rel, req = key.split("|")
    path = os.path.join(REF, rel)
    if not os.path.exists(path):
        pytest.skip("reference assets not present")
    g = GOLD[key]
    px, comp = capi.image_load(path, int(req))
    assert (px.shape[1], px.shape[0], comp) == (g["x"], g["y"], g["comp"])
    b = px.tobytes()
    assert len(b) == g["bytes"]
    assert zlib.crc32(b) & 0xFFFFFFFF == g["crc32"]
    assert hashlib.sha256(b).hexdigest() == g["sha256"]


# ----------------------------------------------------------------- PNG writer
def _chunk(t, d):
    return struct.pack(">I", len(d)) + t + d + struct.pack(">I", zlib.crc32(t + d) & 0xFFFFFFFF)


def _paeth(a, b, c):
    p = a + b - c
    pa, pb, pc = abs(p - a), abs(p - b), abs(p - c)
    return a if pa <= pb and pa <= pc else (b if pb <= pc else c)


def _filter_rows(rows, bpp, rng):
    """rows: list of bytes (raw scanlines); returns filtered stream with random
    filter types (exercises the decoder's unfiltering)."""
    out = bytearray()
    prev = bytes(len(rows[0])) if rows else b""
    for r in rows:
        ft = int(rng.integers(0, 5))
        f = bytearray(len(r))
        for i in range(len(r)):
            a = r[i - bpp] if i >= bpp else 0
            b = prev[i]
            c = prev[i - bpp] if i >= bpp else 0
            pred = [0, a, b, (a + b) >> 1, _paeth(a, b, c)][ft]
            f[i] = (r[i] - pred) & 255
        out.append(ft)
        out += f
        prev = r
    return bytes(out)


def _pack_samples(vals, depth):
    """one scanline of samples -> bytes (big-endian, MSB-first for <8 bits)"""
    if depth == 16:
        return b"".join(struct.pack(">H", int(v)) for v in vals)
    if depth == 8:
        return bytes(int(v) for v in vals)
    bits = "".join(format(int(v), f"0{depth}b") for v in vals)
    bits += "0" * (-len(bits) % 8)
    return bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8))


ADAM7 = [(0, 0, 8, 8), (4, 0, 8, 8), (0, 4, 4, 8), (2, 0, 4, 4), (0, 2, 2, 4), (1, 0, 2, 2), (0, 1, 1, 2)]


def make_png(samples, color, depth, interlace=False, plte=None, trns=None, seed=0):
    """samples: int array [h, w, channels] of raw sample values."""
    rng = np.random.default_rng(seed)
    h, w, ch = samples.shape
    bpp = max(1, ch * depth // 8)
    ihdr = struct.pack(">IIBBBBB", w, h, depth, color, 0, 0, 1 if interlace else 0)
    passes = ADAM7 if interlace else [(0, 0, 1, 1)]
    raw = b""
    for x0, y0, dx, dy in passes:
        sub = samples[y0::dy, x0::dx]
        if sub.shape[0] == 0 or sub.shape[1] == 0:
            continue
        rows = [_pack_samples(sub[y].reshape(-1), depth) for y in range(sub.shape[0])]
        raw += _filter_rows(rows, bpp, rng)
    png = b"\x89PNG\r\n\x1a\n" + _chunk(b"IHDR", ihdr)
    if plte is not None:
        png += _chunk(b"PLTE", bytes(np.asarray(plte, np.uint8).reshape(-1)))
    if trns is not None:
        png += _chunk(b"tRNS", trns)
    # split IDAT in two chunks (decoders must concatenate)
    z = zlib.compress(raw)
    return png + _chunk(b"IDAT", z[: len(z) // 2]) + _chunk(b"IDAT", z[len(z) // 2:]) + _chunk(b"IEND", b"")


def _load_bytes(tmp_path, name, data, req=0):
    p = tmp_path / name
    p.write_bytes(data)
    return capi.image_load(str(p), req)


SCALE = {1: 255, 2: 0x55, 4: 0x11, 8: 1}


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("depth", [1, 2, 4, 8, 16])
def test_png_gray(tmp_path, depth, interlace):
    rng = np.random.default_rng(depth)
    s = rng.integers(0, 2 ** depth, size=(13, 11, 1))
    px, comp = _load_bytes(tmp_path, "g.png", make_png(s, 0, depth, interlace))
    exp = (s >> 8) if depth == 16 else s * SCALE[depth]
    assert comp == 1 and px.shape == (13, 11, 1)
    np.testing.assert_array_equal(px, exp.astype(np.uint8))


@pytest.mark.parametrize("interlace", [False, True])
@pytest.mark.parametrize("color,ch", [(2, 3), (4, 2), (6, 4)])
@pytest.mark.parametrize("depth", [8, 16])
def test_png_truecolor_alpha(tmp_path, color, ch, depth, interlace):
    rng = np.random.default_rng(color * 100 + depth)
    s = rng.integers(0, 2 ** depth, size=(9, 17, ch))
    px, comp = _load_bytes(tmp_path, "c.png", make_png(s, color, depth, interlace))
    exp = (s >> 8) if depth == 16 else s
    assert comp == ch
    np.testing.assert_array_equal(px, exp.astype(np.uint8))


@pytest.mark.parametrize("depth", [1, 2, 4, 8])
def test_png_palette_and_trns(tmp_path, depth):
    rng = np.random.default_rng(depth + 7)
    npal = 2 ** depth
    pal = rng.integers(0, 256, size=(npal, 3))
    s = rng.integers(0, npal, size=(10, 12, 1))
    px, comp = _load_bytes(tmp_path, "p.png", make_png(s, 3, depth, plte=pal))
    assert comp == 3
    np.testing.assert_array_equal(px, pal[s[..., 0]].astype(np.uint8))
    alpha = rng.integers(0, 256, size=npal)
    px, comp = _load_bytes(tmp_path, "pt.png", make_png(s, 3, depth, plte=pal, trns=bytes(alpha.astype(np.uint8))))
    assert comp == 4
    np.testing.assert_array_equal(px[..., :3], pal[s[..., 0]].astype(np.uint8))
    np.testing.assert_array_equal(px[..., 3], alpha[s[..., 0]].astype(np.uint8))


def test_png_color_key(tmp_path):
    rng = np.random.default_rng(3)
    s = rng.integers(0, 4, size=(8, 8, 3)) * 60
    key = (60, 120, 0)
    s[2, 3] = key
    px, comp = _load_bytes(tmp_path, "k.png", make_png(s, 2, 8, trns=struct.pack(">HHH", *key)))
    assert comp == 4
    hit = (s == key).all(-1)
    np.testing.assert_array_equal(px[..., 3], np.where(hit, 0, 255))
    np.testing.assert_array_equal(px[..., :3], s.astype(np.uint8))


def test_png_req_comp_conversions(tmp_path):
    rng = np.random.default_rng(5)
    s = rng.integers(0, 256, size=(6, 7, 3))
    data = make_png(s, 2, 8)
    y = ((s[..., 0] * 77 + s[..., 1] * 150 + s[..., 2] * 29) >> 8).astype(np.uint8)
    px, comp = _load_bytes(tmp_path, "r.png", data, 1)
    assert comp == 3 and px.shape == (6, 7, 1)
    np.testing.assert_array_equal(px[..., 0], y)
    px, _ = _load_bytes(tmp_path, "r.png", data, 4)
    np.testing.assert_array_equal(px[..., :3], s.astype(np.uint8))
    assert (px[..., 3] == 255).all()
    px, _ = _load_bytes(tmp_path, "r.png", data, 2)
    np.testing.assert_array_equal(px[..., 0], y)
    assert (px[..., 1] == 255).all()


def test_write_png_round_trip(tmp_path):
    rng = np.random.default_rng(11)
    img = rng.integers(0, 256, size=(23, 31, 3), dtype=np.uint8)
    p = tmp_path / "o.png"
    capi.write_png(str(p), 31, 23, img)
    px, comp = capi.image_load(str(p))
    assert comp == 3
    np.testing.assert_array_equal(px, img)


# ------------------------------------------------------------------------ TGA
def make_tga(px, rle=False, top_left=False, gray=False):
    h, w, ch = px.shape
    typ = (3 if gray else 2) + (8 if rle else 0)
    bits = 8 if gray else 8 * ch
    hdr = struct.pack("<BBBHHBHHHHBB", 0, 0, typ, 0, 0, 0, 0, 0, w, h, bits, 0x20 if top_left else 0)
    rows = px if top_left else px[::-1]
    flat = rows.reshape(-1, ch)
    if not gray:
        flat = flat[:, [2, 1, 0, 3][:ch]]  # RGB(A) -> BGR(A)
    if not rle:
        return hdr + flat.astype(np.uint8).tobytes()
    out = bytearray()
    i = 0
    n = flat.shape[0]
    while i < n:  # alternate: a repeat packet if the next pixels repeat, else a raw packet
        j = i
        while j + 1 < n and j - i < 127 and (flat[j + 1] == flat[i]).all():
            j += 1
        if j > i:
            out.append(0x80 | (j - i))
            out += flat[i].astype(np.uint8).tobytes()
            i = j + 1
        else:
            k = min(n, i + 5)
            out.append(k - i - 1)
            out += flat[i:k].astype(np.uint8).tobytes()
            i = k
    return hdr + bytes(out)


@pytest.mark.parametrize("rle", [False, True])
@pytest.mark.parametrize("top_left", [False, True])
@pytest.mark.parametrize("ch", [1, 3, 4])
def test_tga(tmp_path, rle, top_left, ch):
    rng = np.random.default_rng(ch * 4 + rle * 2 + top_left)
    px = rng.integers(0, 3, size=(9, 14, ch)).astype(np.uint8) * 100  # runs for RLE
    got, comp = _load_bytes(tmp_path, "t.tga", make_tga(px, rle, top_left, gray=ch == 1))
    assert comp == ch
    np.testing.assert_array_equal(got, px)


# ------------------------------------------------------------------------ BMP
def make_bmp(px, top_down=False, palette=None, idx=None):
    if palette is not None:
        h, w = idx.shape
        bpp, ncol = 8, len(palette)
        rows = [bytes(idx[y].astype(np.uint8)) for y in range(h)]
    else:
        h, w, _ = px.shape
        bpp, ncol = 24, 0
        rows = [px[y][:, ::-1].astype(np.uint8).tobytes() for y in range(h)]
    stride = (w * bpp // 8 + 3) & ~3
    rows = [r + bytes(stride - len(r)) for r in rows]
    if not top_down:
        rows = rows[::-1]
    pal = b"" if palette is None else b"".join(bytes([b, g, r, 0]) for r, g, b in palette)
    off = 14 + 40 + len(pal)
    info = struct.pack("<IiiHHIIiiII", 40, w, -h if top_down else h, 1, bpp, 0, stride * h, 2835, 2835, ncol, 0)
    return b"BM" + struct.pack("<IHHI", off + stride * h, 0, 0, off) + info + pal + b"".join(rows)


@pytest.mark.parametrize("top_down", [False, True])
def test_bmp_24(tmp_path, top_down):
    rng = np.random.default_rng(9)
    px = rng.integers(0, 256, size=(7, 5, 3), dtype=np.uint8)
    got, comp = _load_bytes(tmp_path, "b.bmp", make_bmp(px, top_down))
    assert comp == 3
    np.testing.assert_array_equal(got, px)


def test_bmp_palette(tmp_path):
    rng = np.random.default_rng(10)
    pal = [tuple(int(v) for v in rng.integers(0, 256, 3)) for _ in range(16)]
    idx = rng.integers(0, 16, size=(6, 9))
    got, comp = _load_bytes(tmp_path, "p.bmp", make_bmp(None, palette=pal, idx=idx))
    assert comp == 3
    np.testing.assert_array_equal(got, np.array(pal, np.uint8)[idx])


# --------------------------------------------------------------- error paths
def test_errors(tmp_path):
    with pytest.raises(capi.SrrError):
        capi.image_load(str(tmp_path / "missing.png"))
    bad = tmp_path / "bad.bin"
    bad.write_bytes(b"not an image at all")
    with pytest.raises(capi.SrrError):
        capi.image_load(str(bad))
    trunc = tmp_path / "trunc.png"
    trunc.write_bytes(make_png(np.zeros((4, 4, 3), int), 2, 8)[:40])
    with pytest.raises(capi.SrrError):
        capi.image_load(str(trunc))


def test_image_texture_file_channels(tmp_path):
    """srr_image_texture_file takes RGB/RGBA files (image_texture reads 3 bytes
    per texel) and refuses 1-channel images it would read past."""
    L = capi.lib()
    L.srr_scene_create.restype = ctypes.c_void_p
    L.srr_image_texture_file.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    L.srr_scene_destroy.argtypes = [ctypes.c_void_p]
    s = L.srr_scene_create()
    try:
        rgb = tmp_path / "rgb.png"
        rgb.write_bytes(make_png(np.full((4, 4, 4), 7), 6, 8))
        assert L.srr_image_texture_file(s, str(rgb).encode()) >= 0
        gray = tmp_path / "gray.png"
        gray.write_bytes(make_png(np.full((4, 4, 1), 7), 0, 8))
        assert L.srr_image_texture_file(s, str(gray).encode()) < 0
        assert L.srr_image_texture_file(s, str(tmp_path / "nope.png").encode()) < 0
    finally:
        L.srr_scene_destroy(s)
