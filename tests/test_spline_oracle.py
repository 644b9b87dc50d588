"""CPU checks of the spline3 oracle (oracle/spline_oracle.c).  Parity with the reference is
UNPINNED (no reference test, fixture or wired pipeline exists for spline3); these are the
properties the restated algorithm must have."""
import numpy as np
import pytest

from cusz_amd import datagen


@pytest.mark.parametrize("dims,dtype", [((64, 32, 16), np.float64), ((70, 19, 13), np.float32),
                                        ((45, 37, 1), np.float64), ((300, 1, 1), np.float32)])
def test_roundtrip_error_bound(oracle, dims, dtype):
    x = datagen.smooth3d_np(dims, seed=7, dtype=dtype)
    eb = 1e-4
    c, a, ov, oi = oracle.spline3_c(x, dims, eb)
    y = oracle.spline3_x(c, a, ov, oi, dims, eb)
    assert np.max(np.abs(y.astype(np.float64) - x)) <= 1.001 * eb


def test_anchors_are_lattice_values(oracle):
    dims = (70, 19, 13)
    x = datagen.smooth3d_np(dims, seed=3)
    _, a, _, _ = oracle.spline3_c(x, dims, 1e-3)
    v = x.reshape(dims[2], dims[1], dims[0])[::8, ::8, ::8]
    np.testing.assert_array_equal(a, v.ravel())


def test_tile_independence(oracle):
    """Codes of a tile depend only on its 33x9x9 region (spline3.cu:29 tiling)."""
    dims = (96, 24, 24)
    x = datagen.smooth3d_np(dims, seed=4, dtype=np.float64)
    c0, _, _, _ = oracle.spline3_c(x, dims, 1e-5)
    y = x.reshape(24, 24, 96).copy()
    y[17:, :, :] += 0.5          # beyond the z = 0..8 region of the first tile layer
    y[:, :, 41:] -= 0.25         # beyond x = 0..32 of the first tile column
    c1, _, _, _ = oracle.spline3_c(y.ravel(), dims, 1e-5)
    a = c0.reshape(24, 24, 96)[:8, :8, :32]
    b = c1.reshape(24, 24, 96)[:8, :8, :32]
    np.testing.assert_array_equal(a, b)


def test_outlier_order_and_codes(oracle):
    dims = (70, 19, 13)
    x = datagen.smooth3d_np(dims, seed=5)
    eb = 1e-6
    c, _, ov, oi = oracle.spline3_c(x, dims, eb)
    assert len(oi) > 100
    assert np.all(c[oi] == 0)
    gx, gy, gz = oi % 70, (oi // 70) % 19, oi // (70 * 19)
    tile = gx // 32 + 3 * (gy // 8 + 3 * (gz // 8))
    key = tile.astype(np.int64) * 4096 + (gz % 8) * 512 + (gy % 8) * 32 + gx % 32
    assert np.all(np.diff(key) > 0)
    assert np.all((ov < 0) | (ov >= 1024))  # outliers are exactly the codes outside [0, 2r)
