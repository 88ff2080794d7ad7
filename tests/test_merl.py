"""MERL measured-BRDF lookup (brdf.h): the product's lookup
(include/srr/merl.h through srr_merl_* on the device, and the same header built
for the host) against the reference's own std_coords_to_half_diff_coords +
lookup_brdf_val as compiled HERE (oracle/ref: g++ -O2, glibc 2.35, FMA ifunc
variants; the reference ships as an MSVC project whose UCRT libm is another
implementation, so for out == in the pin is to this oracle port and parity with
the MSVC build is unpinned) on a synthetic 90x90x180x3 table (the measured
.binary files are not shipped with the reference):

* tests/golden/kat_merl.bin: random (in, out) angle pairs, every 5th with
  out == in, every 7th with theta_in = 0 (oracle/ref kat.inc "merl");
* tests/golden/kat_merl_same.bin: brdfmaterial::scatter's own call pattern,
  theta_in / phi_in derived from a random direction and normal as scatter does
  and out == in on every record (material.h:214-231, kat.inc "merl_same").

Bar: the table cell and the scaled RGB doubles bit-identical on EVERY record.
out == in is the ill-conditioned case -- the difference vector is (0, 0, 1) up
to ~1e-17 residues and phi_diff = atan2(residue, residue) -- so it holds only
because the lookup runs glibc's own dbl-64 cos / sin / acos / atan2
(include/srr/glibc_math64.h, checked against libm by tools/check_glibc_math64.cpp)."""
import os
import shutil
import subprocess

import numpy as np
import pytest

import oracle_bind as ob
from srr import capi

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def synthetic_table() -> np.ndarray:
    """oracle/ref/kat.inc merl_table(): ((k * 2654435761) mod 1000003) / 1000, -1 every 97th."""
    k = np.arange(3 * capi.MERL_CELLS, dtype=np.uint64)
    t = ((k * np.uint64(2654435761)) % np.uint64(1000003)).astype(np.float64) / 1000.0
    t[(k % np.uint64(97)) == 0] = -1.0
    return t


def kat_f64(chunks: np.ndarray) -> np.ndarray:
    """Three exact 24-bit float chunks per double (kat.inc push_f64) -> float64."""
    c = chunks.astype(np.uint64).reshape(-1, 3)
    return (c[:, 0] | (c[:, 1] << np.uint64(24)) | (c[:, 2] << np.uint64(48))).view(np.float64)


def kat(name):
    rec = ob.read_kat(name)
    return (rec[:, :4].astype(np.float64), rec[:, 4].astype(np.int64), kat_f64(rec[:, 9:18]).reshape(-1, 3),
            (rec[:, 0] == rec[:, 2]) & (rec[:, 1] == rec[:, 3]))


def check(name, cell, rgb, want_cell, want_rgb):
    bad = np.flatnonzero(cell != want_cell)
    assert len(bad) == 0, f"{name}: {len(bad)} cells differ, first {bad[:5]}: {cell[bad[:5]]} vs {want_cell[bad[:5]]}"
    np.testing.assert_array_equal(rgb.view(np.uint64), want_rgb.view(np.uint64))


def test_kat_shapes():
    """The sweeps hold the cases they are meant to: out == in on a fifth of the
    random records and on every scatter record, and degenerate cells that are
    not the trivial phi_diff 0 (the residues' atan2 lands in many cells)."""
    _, c1, _, deg1 = kat("merl")
    _, c2, _, deg2 = kat("merl_same")
    assert deg1.sum() >= len(deg1) // 6 and (~deg1).sum() > len(deg1) // 2
    assert deg2.all() and len(deg2) == 4096
    assert len(np.unique(c2 % 180)) > 20


def test_merl_kats_record_their_libm():
    """The KATs' libm is recorded (tests/golden/make_golden.py refuses to
    regenerate them on another glibc or without the FMA ifunc variants)."""
    import json
    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))
    assert meta["merl_libm"] == {"glibc": "glibc 2.35", "fma_ifunc": True}


def test_merl_host_build_matches_reference(tmp_path):
    """merl.h + glibc_math64.h built for the host (g++, as the reference's host
    code is) against both KATs: every cell and RGB bit-identical."""
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("no g++")
    exe = tmp_path / "merl_host"
    subprocess.run([gxx, "-std=c++17", "-O2", "-ffp-contract=off", os.path.join(ROOT, "tests", "cpp", "merl_host.cpp"),
                    "-o", str(exe)], check=True)
    for name in ("merl", "merl_same"):
        ang, want_cell, want_rgb, _ = kat(name)
        q, o = tmp_path / f"{name}.in", tmp_path / f"{name}.out"
        ang.tofile(q)
        subprocess.run([str(exe), str(q), str(o)], check=True)
        n = len(ang)
        raw = np.fromfile(o, dtype=np.uint8)
        cell = raw[:4 * n].view(np.int32).astype(np.int64)
        rgb = raw[4 * n:].view(np.float64).reshape(n, 3)
        check(name, cell, rgb, want_cell, want_rgb)


def test_merl_load_rejects_wrong_dimensions(tmp_path):
    """brdf::read_brdf's dimension check (brdf.h:170-176): no GPU needed, the
    header is checked before anything is uploaded."""
    p = tmp_path / "bad.binary"
    np.array([90, 90, 90], np.int32).tofile(p)
    with pytest.raises(capi.SrrError, match="dimensions"):
        capi.Merl.load(str(p))


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["merl", "merl_same"])
def test_merl_lookup_matches_reference(name, tmp_path):
    """The device lookup (k_merl_lookup through srr_merl_lookup): every record's
    cell and RGB bit-identical, out == in included."""
    ang, want_cell, want_rgb, deg = kat(name)
    m = capi.Merl(synthetic_table())
    rgb, cell = m.lookup(ang)
    check(name, cell, rgb, want_cell, want_rgb)
    print(f"{name}: {len(ang)} queries ({deg.sum()} with out == in), all in the reference's cell")
    if name == "merl":
        # the file path (read_brdf) gives the same table
        p = tmp_path / "synthetic.binary"
        with open(p, "wb") as f:
            np.array([90, 90, 180], np.int32).tofile(f)
            synthetic_table().tofile(f)
        rgb2, cell2 = capi.Merl.load(str(p)).lookup(ang)
        np.testing.assert_array_equal(rgb2.view(np.uint64), rgb.view(np.uint64))
        np.testing.assert_array_equal(cell2, cell)
