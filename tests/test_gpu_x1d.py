"""1-D reconstruction reading the outlier values straight from the archive's cells: the
reference layout's k_lorenzo_x1d (X1dOutliers, per 16384-element brick) and the fused 1-D brick
decoder (brick.hip k_brick1_decode, per chunk).  Sorted cells (no spill) take that path, cells
with a spill tail (one brick over its slot) fall back to the scatter.  Both must equal the
oracle's decompression bit for bit (run_roundtrip), and a shuffled cell list must decompress
identically.
"""
import numpy as np
import pytest

from gpu_util import d2h, empty_device, parse_archive, sync, to_device
from test_gpu_parity import run_roundtrip

import cusz_amd as cz

pytestmark = pytest.mark.gpu


def _walk(n, seed, jump_frac=0.05, burst=None):
    rng = np.random.default_rng(seed)
    x = np.cumsum(rng.standard_normal(n)).astype(np.float32)
    j = rng.random(n) < jump_frac
    x[j] += rng.standard_normal(j.sum()).astype(np.float32) * 400
    if burst is not None:  # one 16384-element brick far past its 10 % outlier slot
        a, b = burst
        x[a:b] += rng.standard_normal(b - a).astype(np.float32) * 100
    return x


LAYOUTS = [cz.LAYOUT_BRICK, cz.LAYOUT_REFERENCE]


@pytest.mark.parametrize("layout", LAYOUTS, ids=["brick", "reference"])
@pytest.mark.parametrize("n,burst", [(300_001, None), (16384 * 3 + 77, None), (200_000, (40_000, 50_000)),
                                     (16384, None)])
def test_x1d_outliers_match_oracle(oracle, n, burst, layout):
    data = _walk(n, n, burst=burst)
    run_roundtrip(oracle, data, (n, 1, 1), 0.05, layout=layout)


@pytest.mark.parametrize("layout", LAYOUTS, ids=["brick", "reference"])
def test_x1d_shuffled_cells_decompress_identically(layout):
    import torch

    n = 100_000
    data = _walk(n, 7)
    r = cz.Resource(cz.F4, (n, 1, 1))
    r.set_layout(layout)
    d_in = to_device(data)
    ptr, nbytes, _ = r.compress(d_in.data_ptr(), 0.05, cz.Abs)
    arch = bytearray(d2h(ptr, nbytes).tobytes())
    out0 = empty_device(n, torch.float32)
    r.decompress(ptr, nbytes, out0.data_ptr())
    sync()
    h = parse_archive(bytes(arch))["header"]
    cells = np.frombuffer(bytes(arch[h.entry[3]:h.entry[4]]), np.uint64).copy()
    assert cells.size > 1000
    arch[h.entry[3]:h.entry[4]] = cells[np.random.default_rng(3).permutation(cells.size)].tobytes()
    d_arch = torch.tensor(np.frombuffer(bytes(arch), np.uint8)).cuda()
    out1 = empty_device(n, torch.float32)
    r.decompress(d_arch.data_ptr(), nbytes, out1.data_ptr())
    sync()
    np.testing.assert_array_equal(out1.cpu().numpy().view(np.uint32), out0.cpu().numpy().view(np.uint32))
    r.close()
