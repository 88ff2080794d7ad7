"""MERL measured-BRDF lookup (brdf.h): the device lookup
(csrc/merl.h through srr_merl_*) against the REFERENCE's own
std_coords_to_half_diff_coords + lookup_brdf_val (tests/golden/kat_merl.bin, made
by oracle/ref from brdf.h) on a synthetic 90x90x180x3 table -- the measured
.binary files are not shipped with the reference.  Table cells must be equal and
the scaled RGB doubles bit-identical (see the test for the one ill-conditioned
case, out == in)."""
import numpy as np
import pytest

import oracle_bind as ob
from srr import capi


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


def test_merl_load_rejects_wrong_dimensions(tmp_path):
    """brdf::read_brdf's dimension check (brdf.h:170-176): no GPU needed, the
    header is checked before anything is uploaded."""
    p = tmp_path / "bad.binary"
    np.array([90, 90, 90], np.int32).tofile(p)
    with pytest.raises(capi.SrrError, match="dimensions"):
        capi.Merl.load(str(p))


@pytest.mark.gpu
def test_merl_lookup_matches_reference(tmp_path):
    """Bit-exact on every well-conditioned query.  When the outgoing direction
    equals the incoming one (brdfmaterial's own call, material.h:231; every 5th
    KAT record) the difference vector is (0, 0, 1) up to ~1e-17 residues and
    phi_diff = atan2(residue, residue) is decided by the last-ulp rounding of the
    double cos / sin / acos / atan2 calls, which glibc and the device libm (ocml)
    do not share: there the theta_half and theta_diff cells must still agree, the
    phi_diff cell (and the value read there) is parity unpinned."""
    rec = ob.read_kat("merl")
    angles = rec[:, :4].astype(np.float64)
    m = capi.Merl(synthetic_table())
    rgb, cell = m.lookup(angles)
    want_cell = rec[:, 4].astype(np.int64)
    want_rgb = kat_f64(rec[:, 9:18]).reshape(-1, 3)
    degenerate = (rec[:, 0] == rec[:, 2]) & (rec[:, 1] == rec[:, 3])
    assert degenerate.sum() >= len(rec) // 6 and (~degenerate).sum() > len(rec) // 2
    ok = ~degenerate
    bad = np.flatnonzero(ok & (cell != want_cell))
    assert len(bad) == 0, f"{len(bad)} cells differ, first {bad[:5]}: dev {cell[bad[:5]]} ref {want_cell[bad[:5]]}"
    np.testing.assert_array_equal(rgb[ok].view(np.uint64), want_rgb[ok].view(np.uint64))
    np.testing.assert_array_equal(cell[degenerate] // 180, want_cell[degenerate] // 180)  # theta_half, theta_diff
    same = degenerate & (cell == want_cell)
    np.testing.assert_array_equal(rgb[same].view(np.uint64), want_rgb[same].view(np.uint64))
    print(f"degenerate queries: {same.sum()} of {degenerate.sum()} in the reference's phi_diff cell")
    # the file path (read_brdf) gives the same table
    p = tmp_path / "synthetic.binary"
    with open(p, "wb") as f:
        np.array([90, 90, 180], np.int32).tofile(f)
        synthetic_table().tofile(f)
    rgb2, cell2 = capi.Merl.load(str(p)).lookup(angles)
    np.testing.assert_array_equal(rgb2.view(np.uint64), rgb.view(np.uint64))
    np.testing.assert_array_equal(cell2, cell)
