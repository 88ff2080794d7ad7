"""image_texture::value divides each byte by 255 in double and rounds the quotient to
float (texture.h:66-68: `int(data[..]) / 255.0`); kernels.hip tex_value_slow divides in
float instead.  Exact for every byte value: double rounding (exact -> double -> float) never
differs from the direct float rounding here."""
import numpy as np


def test_float_quotient_equals_the_double_one_for_every_byte():
    x = np.arange(256)
    via_double = (x.astype(np.float64) / 255.0).astype(np.float32)
    direct = x.astype(np.float32) / np.float32(255.0)
    assert direct.dtype == np.float32
    np.testing.assert_array_equal(via_double.view(np.uint32), direct.view(np.uint32))
