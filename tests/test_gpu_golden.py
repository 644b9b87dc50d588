"""The GPU path against fixtures produced by the compiled reference itself (tests/golden,
make_golden.py): Lorenzo-3D f32, its ZigZag instantiation (lrz.seq.cc:82) and the 3-D template
for double, integer data at eb = 0.5 (where the reference CPU path and the GPU semantics
coincide).  Also the HACC-like outlier stress of SURVEY §8d config 3."""
import os

import numpy as np
import pytest
import torch

import cusz_amd as cz
from cusz_amd import datagen
from gpu_util import d2h, parse_archive, sync, to_device

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("fixture,zigzag", [("ref_lrz3d.npz", False), ("ref_lrz3d_zz.npz", True),
                                            ("ref_lrz3d_f64.npz", False)])
def test_gpu_matches_reference_fixture(fixture, zigzag):
    g = np.load(os.path.join(GOLDEN, fixture))
    dims = tuple(int(v) for v in g["dims"])
    data = g["data"]
    f64 = data.dtype == np.float64
    r = cz.Resource(cz.F8 if f64 else cz.F4, dims, cz.LorenzoZigZag if zigzag else cz.Lorenzo)
    d = to_device(data)
    ptr, nb, _ = r.compress(d.data_ptr(), 0.5)
    arch = d2h(ptr, nb).tobytes()
    r.decode_codes(ptr)
    sync()
    codes = d2h(r.internals().d_quant_codes, 2 * data.size, np.uint16)
    np.testing.assert_array_equal(codes, g["codes"])
    a = parse_archive(arch)
    order = np.argsort(a["ol_idx"], kind="stable")
    ref_order = np.argsort(g["ol_idx"], kind="stable")
    np.testing.assert_array_equal(a["ol_idx"][order], g["ol_idx"][ref_order])
    np.testing.assert_array_equal(a["ol_val"][order], g["ol_val"][ref_order])
    out = torch.full((data.size,), float("nan"), dtype=torch.float64 if f64 else torch.float32, device="cuda")
    r.decompress(ptr, nb, out.data_ptr())
    sync()
    np.testing.assert_array_equal(out.cpu().numpy(), data)


def test_hacc_jump_stress_beyond_cap_grows(oracle):
    """30 % uniform jumps: more outliers than the reference's 10 % cap (buf_comp.cc:87-88, where
    compressor.inl:368-372 gives up).  Here the outlier capacity grows: the archive is valid,
    holds every outlier (the oracle's set and values) and decompresses within the bound."""
    n = 4_000_000
    d = datagen.hacc1d_torch(n, seed=7, jump=0.30)
    r = cz.Resource(cz.F4, (n, 1, 1))
    ptr, nb, st = r.compress(d.data_ptr(), 1e-4)
    assert st == cz.PSZ_SUCCESS
    a = parse_archive(d2h(ptr, nb).tobytes())
    host = d.cpu().numpy()
    codes, ov, oi = oracle.lorenzo_c(host, (n, 1, 1), 1e-4)
    assert a["header"].splen == len(oi) > n // 10
    order = np.argsort(a["ol_idx"], kind="stable")
    np.testing.assert_array_equal(a["ol_idx"][order], oi)
    np.testing.assert_array_equal(a["ol_val"][order].view(np.uint32), ov.view(np.uint32))
    out = torch.empty(n, dtype=torch.float32, device="cuda")
    r.decompress(ptr, nb, out.data_ptr())
    sync()
    xg = out.cpu().numpy()
    np.testing.assert_array_equal(xg, oracle.lorenzo_x(codes, ov, oi, (n, 1, 1), 1e-4))
    assert np.abs(xg.astype(np.float64) - host).max() <= 1e-4 * 1.001 + 256 * 2.0 ** -23


def test_hacc_jump_within_cap_roundtrip():
    n = 4_000_011  # n mod 1024 != 0: partial last tile
    d = datagen.hacc1d_torch(n, seed=8, jump=0.05)
    r = cz.Resource(cz.F4, (n, 1, 1))
    ptr, nb, st = r.compress(d.data_ptr(), 1e-4)
    assert st == cz.PSZ_SUCCESS
    assert r.header.splen > 0.04 * n
    out = torch.empty(n, device="cuda")
    r.decompress(ptr, nb, out.data_ptr())
    sync()
    err = (out.double() - d.double()).abs().max().item()
    assert err <= 1.001e-4 + 2.0 ** -23 * 256
