"""Pin the CPU oracle (oracle/psz_oracle.c) before trusting it (CPU-only).

Fixtures under tests/golden/ are the reference's own KATs (correctness.inl) and
outputs of the compiled reference CPU path; see tests/golden/make_golden.py.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

R = 512


def _kat():
    return np.load(os.path.join(GOLDEN, "kat_lorenzo.npz"))


@pytest.mark.parametrize("t,dims", [("t1", (256, 1, 1)), ("t2", (16, 16, 1)), ("t3", (8, 8, 8))])
def test_kat_compress(oracle, t, dims):
    """test/src/test_lrz.seq.cc test1: all-ones input, eb=0.5 -> codes = delta + radius."""
    k = _kat()
    codes, ov, oi = oracle.lorenzo_c(k[f"{t}_in"], dims, eb=0.5)
    np.testing.assert_array_equal(codes.astype(np.float32), k[f"{t}_comp_out"] + R)
    assert len(oi) == 0


@pytest.mark.parametrize("t,dims", [("t1", (256, 1, 1)), ("t2", (16, 16, 1)), ("t3", (8, 8, 8))])
def test_kat_decompress(oracle, t, dims):
    """test2: codes = t_eq + radius, eb=0.5 (ebx2 = 1) -> tile prefix sums."""
    k = _kat()
    codes = (k[f"{t}_eq"].astype(np.int32) + R).astype(np.uint16)
    out = oracle.lorenzo_x(codes, [], [], dims, eb=0.5)
    np.testing.assert_array_equal(out, k[f"{t}_decomp_out"])


@pytest.mark.parametrize("t,dims", [("t1", (256, 1, 1)), ("t2", (16, 16, 1)), ("t3", (8, 8, 8))])
def test_kat_roundtrip(oracle, t, dims):
    k = _kat()
    codes, ov, oi = oracle.lorenzo_c(k[f"{t}_in"], dims, eb=0.5)
    out = oracle.lorenzo_x(codes, ov, oi, dims, eb=0.5)
    np.testing.assert_array_equal(out, k[f"{t}_in"])


def test_ref_lorenzo3d_integer_crosscheck(oracle):
    """Compiled reference CPU Lorenzo-3D on integer data at eb=0.5 (8^3 tiles coincide)."""
    g = np.load(os.path.join(GOLDEN, "ref_lrz3d.npz"))
    dims = tuple(int(v) for v in g["dims"])
    codes, ov, oi = oracle.lorenzo_c(g["data"], dims, eb=0.5)
    np.testing.assert_array_equal(codes, g["codes"])
    order = np.argsort(g["ol_idx"], kind="stable")
    np.testing.assert_array_equal(oi, g["ol_idx"][order])
    np.testing.assert_array_equal(ov, g["ol_val"][order])
    out = oracle.lorenzo_x(codes, ov, oi, dims, eb=0.5)
    np.testing.assert_array_equal(out, g["data"])


@pytest.mark.parametrize("fixture,zigzag", [("ref_lrz3d_zz.npz", True), ("ref_lrz3d_f64.npz", False)])
def test_ref_lorenzo3d_zigzag_f64_crosscheck(oracle, fixture, zigzag):
    """Compiled reference on integer data at eb=0.5: the ZigZag instantiation (lrz.seq.cc:82) and
    the 3-D template for double (lrz.seq.inl, instantiated by oracle/ref_shim.cc)."""
    g = np.load(os.path.join(GOLDEN, fixture))
    dims = tuple(int(v) for v in g["dims"])
    codes, ov, oi = oracle.lorenzo_c(g["data"], dims, eb=0.5, zigzag=zigzag)
    np.testing.assert_array_equal(codes, g["codes"])
    order = np.argsort(g["ol_idx"], kind="stable")
    np.testing.assert_array_equal(oi, g["ol_idx"][order])
    np.testing.assert_array_equal(ov, g["ol_val"][order])
    out = oracle.lorenzo_x(codes, ov, oi, dims, eb=0.5, zigzag=zigzag, dtype=g["data"].dtype)
    np.testing.assert_array_equal(out, g["data"])


@pytest.mark.parametrize("zigzag", [False, True])
def test_ref_ragged_dense_outliers(oracle, zigzag):
    """The compiled reference on a ragged field where almost every point is an outlier: its
    outlier list is sized by the padded tile count (pyoracle._ref_outlier_cap), so partial-tile
    appends past the field stay inside the buffer; the in-field part equals the oracle's."""
    from oracle import pyoracle
    if not pyoracle.ref_available():
        pytest.skip("oracle/_ref not built (this container builds it from /root/reference)")
    dims = (40, 24, 17)
    rng = np.random.default_rng(11)
    # integer data at eb = 0.5: the reference CPU kernel does not round, so only integer inputs
    # make its quantization coincide with the oracle's (as in the crosschecks above)
    data = rng.integers(-4000, 4000, size=dims[::-1]).astype(np.float32).ravel()
    fn = pyoracle.ref_lorenzo_c_zz_f32 if zigzag else pyoracle.ref_lorenzo_c_f32
    codes, ov, oi = fn(data, dims, 0.5)
    n = data.size
    assert len(oi) > n // 2
    inside = oi < n
    mine_codes, mine_ov, mine_oi = oracle.lorenzo_c(data, dims, eb=0.5, zigzag=zigzag)
    order = np.argsort(oi[inside], kind="stable")
    np.testing.assert_array_equal(mine_oi, oi[inside][order])
    np.testing.assert_array_equal(mine_ov, ov[inside][order])
    np.testing.assert_array_equal(mine_codes, codes)


def test_ref_histogram(oracle):
    g = np.load(os.path.join(GOLDEN, "ref_hist.npz"))
    np.testing.assert_array_equal(oracle.histogram(g["codes"]), g["hist"])


def test_ref_codebook_bytes(oracle):
    """Oracle codebook == reference phf_CPU_build_canonized_codebook_v2, byte for byte."""
    g = np.load(os.path.join(GOLDEN, "ref_codebook.npz"))
    for h, book, rv in zip(g["hist"], g["book"], g["revbook"]):
        ob, orv = oracle.codebook(h)
        np.testing.assert_array_equal(ob, book)
        np.testing.assert_array_equal(orv, rv)


def test_codebook_single_symbol_deviation(oracle):
    """Reference emits a 0-bit code (undecodable); we define a 1-bit code."""
    h = np.zeros(1024, np.uint32)
    h[512] = 1000
    book, rv = oracle.codebook(h)
    assert book[512] >> 27 == 1
    codes = np.full(1000, 512, np.uint16)
    nbit, entry, bs, tot = oracle.hf_encode(codes, book, 256)
    assert tot == 1000
    dec = oracle.hf_decode(bs, rv, nbit, entry, 256, 1000)
    np.testing.assert_array_equal(dec, codes)


def test_codebook_length_limit(oracle):
    """Fibonacci frequencies deeper than 27 bits are length-limited (reference: broken code)."""
    h = np.zeros(1024, np.uint32)
    a, b = 1, 1
    for i in range(40):
        h[300 + i] = min(a, 2**31)
        a, b = b, a + b
    lens = oracle.huffman_lengths(h)
    assert lens.max() == 27
    used = lens[lens > 0].astype(np.float64)
    assert np.sum(2.0 ** -used) <= 1.0 + 1e-12
    book, rv = oracle.codebook(h)
    rng = np.random.default_rng(0)
    codes = rng.choice(np.arange(300, 340), 5000).astype(np.uint16)
    nbit, entry, bs, tot = oracle.hf_encode(codes, book, 512)
    np.testing.assert_array_equal(oracle.hf_decode(bs, rv, nbit, entry, 512, codes.size), codes)


@pytest.mark.parametrize("n,sublen", [(1, 256), (1000, 256), (70001, 2048), (4096, 4096)])
def test_huffman_roundtrip(oracle, n, sublen):
    rng = np.random.default_rng(n)
    codes = np.clip(rng.normal(512, 9, n).round(), 0, 1023).astype(np.uint16)
    h = oracle.histogram(codes)
    book, rv = oracle.codebook(h)
    nbit, entry, bs, tot = oracle.hf_encode(codes, book, sublen)
    lens = (book[codes] >> 27).astype(np.int64)
    assert tot == lens.sum()
    dec = oracle.hf_decode(bs, rv, nbit, entry, sublen, n)
    np.testing.assert_array_equal(dec, codes)


def test_coarse_tune_mi355x(oracle):
    """libphf.cc:26-70 on MI355X (256 CUs, 1024 threads/block): 512^3 -> 2048 / 65536."""
    assert oracle.coarse_tune(512**3) == (2048, 65536)
    assert oracle.coarse_tune(3600 * 1800) == (256, 25313)


@pytest.mark.parametrize("dims", [(1000, 1, 1), (3000, 1, 1), (70, 45, 1), (33, 17, 9), (16, 16, 16)])
@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("zigzag", [False, True])
def test_error_bound_property(oracle, dims, dtype, zigzag):
    rng = np.random.default_rng(7)
    n = dims[0] * dims[1] * dims[2]
    data = (np.cumsum(rng.normal(0, 0.01, n)) + rng.normal(0, 1e-3, n)).astype(dtype)
    eb = 1e-3
    codes, ov, oi = oracle.lorenzo_c(data, dims, eb, zigzag=zigzag)
    out = oracle.lorenzo_x(codes, ov, oi, dims, eb, zigzag=zigzag, dtype=dtype)
    assert np.max(np.abs(out.astype(np.float64) - data)) <= 1.001 * eb
