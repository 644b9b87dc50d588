"""The 3-D decoder's 32-column mode (12 waves per CU, `recon_block32`), which the launcher picks
for f32 fields of at least 12 bricks per CU (3072 on MI355X): parity needs fields that large.
Each case decompresses through the fused decoder into a NaN-poisoned buffer and must equal the
oracle's reconstruction bit for bit (lrz_x.cuhip.inl:271-360 order).  Ragged y and z extents
exercise the partial bricks, whose rows past the field sit in the upper lane half; spikes give
outliers, ranked per lane half (ZigZag off) or read from the scattered field (ZigZag on)."""
import numpy as np
import pytest
import torch

import cusz_amd as cz
from gpu_util import d2h, empty_device, sync, to_device

pytestmark = pytest.mark.gpu


def _field(dims, seed, spikes):
    x, y, z = dims
    rng = np.random.default_rng(seed)
    xs = np.arange(x, dtype=np.float64)
    ys = np.arange(y, dtype=np.float64)[:, None]
    plane = np.sin(0.05 * xs)[None, :] * np.cos(0.07 * ys)
    out = np.empty((z, y, x), np.float32)
    for k in range(z):
        out[k] = plane + 0.5 * np.sin(0.03 * k + 0.01 * xs)[None, :]
    f = out.ravel()
    f += (1e-3 * rng.standard_normal(f.size)).astype(np.float32)
    if spikes:  # outliers: clustered in some bricks (more cells than a brick stages in LDS)
        idx = rng.choice(f.size, size=spikes, replace=False)
        f[idx] += rng.uniform(-50, 50, size=spikes).astype(np.float32)
        f[: 256 * 8 * 3] += rng.uniform(-50, 50, size=256 * 8 * 3).astype(np.float32)
    return f


@pytest.mark.parametrize("dims,zigzag,spikes", [
    ((512, 500, 196), False, 20000),  # 2 x 63 x 25 = 3150 bricks, partial in y and z
    ((512, 512, 200), True, 5000),    # 3200 bricks, full; ZigZag: outliers from the scatter
    ((768, 504, 132), False, 0),      # 3 x 63 x 17 = 3213 bricks, partial in z only
])
def test_brick32_decoder_bit_exact(oracle, dims, zigzag, spikes):
    data = _field(dims, sum(dims), spikes)
    nbricks = (dims[0] // 256) * -(-dims[1] // 8) * -(-dims[2] // 8)
    assert nbricks >= 12 * 256  # the 32-column mode (on MI355X's 256 CUs)
    eb = 1e-4
    r = cz.Resource(cz.F4, dims, cz.LorenzoZigZag if zigzag else cz.Lorenzo)
    d_in = to_device(data)
    ptr, nbytes, _ = r.compress(d_in.data_ptr(), eb)
    assert r.internals().layout == cz.LAYOUT_BRICK
    codes_o, ov_o, oi_o = oracle.lorenzo_c(data, dims, eb, 512, zigzag)
    if spikes:
        assert oi_o.size > 1000
    xo = oracle.lorenzo_x(codes_o, ov_o, oi_o, dims, eb, 512, zigzag, np.float32)
    out = empty_device(data.size, torch.float32)
    out.fill_(float("nan"))
    r.decompress(ptr, nbytes, out.data_ptr())
    sync()
    xg = out.cpu().numpy()
    bad = np.flatnonzero(xg.view(np.uint32) != xo.view(np.uint32))
    assert bad.size == 0, f"{bad.size} mismatches, first {bad[:5]}: {xg[bad[:5]]} vs {xo[bad[:5]]}"
    r.close()
