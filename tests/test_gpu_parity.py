"""Parity of the HIP product path (through the C-ABI) against the CPU oracle.

Bit-exact: quant codes, outlier set (index + value), histogram, codebook, the whole
Huffman (phf) segment of the archive at the same chunk length, and the decompressed
field (the oracle follows the reference's floating-point operation order).  Outlier
cell ORDER is not compared (the reference's order is nondeterministic; ours is
deterministic brick order) -- cells are compared sorted by index.
"""
import os

import numpy as np
import pytest

import cusz_amd as cz
from cusz_amd import datagen
from gpu_util import check_phf_against_oracle, d2h, expected_books, empty_device, parse_archive, sync, to_device

pytestmark = pytest.mark.gpu


def _field(kind, dims, dtype, seed):
    n = int(np.prod(dims))
    rng = np.random.default_rng(seed)
    if kind == "smooth":
        return datagen.smooth3d_np(dims, seed, dtype=dtype)
    if kind == "walk":
        return datagen.hacc1d_np(n, seed, jump=0.05, dtype=dtype)
    if kind == "int":
        return np.cumsum(rng.integers(-3, 4, n)).astype(dtype)
    if kind == "noise":
        return rng.standard_normal(n).astype(dtype)
    raise ValueError(kind)


def run_roundtrip(oracle, data, dims, eb, dtype=np.float32, zigzag=False, radius=512, sublen=0,
                  check_bound=True, layout=None, codebook=None):
    n = int(np.prod(dims))
    tdt = "float32" if dtype == np.float32 else "float64"
    import torch

    r = cz.Resource(cz.F4 if dtype == np.float32 else cz.F8, dims,
                    cz.LorenzoZigZag if zigzag else cz.Lorenzo)
    if sublen:
        r.set_sublen(sublen)
    if layout is not None:
        r.set_layout(layout)
    if codebook is not None:
        r.set_codebook(codebook)
    d_in = to_device(data)
    ptr, nbytes, st = r.compress(d_in.data_ptr(), eb, cz.Abs, radius)
    arch = d2h(ptr, nbytes).tobytes()
    a = parse_archive(arch)
    h = a["header"]
    assert h.entry[5] == nbytes == len(arch)
    assert (h.len.x, h.len.y, h.len.z) == tuple(dims)

    # ---- stage 1: quant codes and outliers vs oracle --------------------------------------
    ino = r.internals()
    if ino.layout == cz.LAYOUT_BRICK:  # codes never reach HBM: decode them with the general decoder
        assert a["sublen"] == ino.brick_width
        r.decode_codes(ptr)
        sync()
    codes_g = d2h(ino.d_quant_codes, 2 * n, np.uint16)
    codes_o, ov_o, oi_o = oracle.lorenzo_c(data, dims, eb, radius, zigzag)
    mism = np.flatnonzero(codes_g != codes_o)
    assert mism.size == 0, f"{mism.size} code mismatches, first at {mism[:5]}"
    order = np.argsort(a["ol_idx"], kind="stable")
    np.testing.assert_array_equal(a["ol_idx"][order], oi_o)
    np.testing.assert_array_equal(a["ol_val"][order].view(np.uint32), ov_o.view(np.uint32))
    assert h.splen == len(oi_o)

    # ---- stage 2: histogram, codebook, Huffman segment ------------------------------------
    bklen = 2 * radius
    hist_g = d2h(ino.d_hist, 4 * bklen, np.uint32)
    np.testing.assert_array_equal(hist_g, oracle.histogram(codes_o, bklen))
    books = expected_books(oracle, r, codes_o, dims, bklen, ino.layout)
    seg_o, info = oracle.phf_segment(codes_o, bklen, sublen=a["sublen"], books=books)
    check_phf_against_oracle(a, info, seg_o, ino.layout)

    # ---- stage 3: decompress into an un-zeroed, NaN-poisoned buffer, with each decoder -----
    xo = oracle.lorenzo_x(codes_o, ov_o, oi_o, dims, eb, radius, zigzag, dtype)
    ubits = np.uint64 if dtype == np.float64 else np.uint32
    for dec in DECODERS:
        r.set_decoder(dec)
        out = empty_device(n, getattr(torch, tdt))
        out.fill_(float("nan"))
        r.decompress(ptr, nbytes, out.data_ptr())
        sync()
        xg = out.cpu().numpy()
        bad = np.flatnonzero(xg.view(ubits) != xo.view(ubits))
        assert bad.size == 0, f"decoder {dec}: {bad.size} reconstruction mismatches, first {bad[:5]}: " \
                              f"{xg[bad[:5]]} vs {xo[bad[:5]]}"
    r.set_decoder(cz.DECODER_AUTO)
    if check_bound:  # f32/f64 prequant rounding adds a few ulp of |x| (same in the reference)
        tol = 1.001 * eb + 4 * float(np.spacing(np.abs(data).max().astype(dtype)))
        assert np.max(np.abs(xg.astype(np.float64) - data)) <= tol
    r.close()
    return arch, a


# auto, one lane per chunk, one wave per chunk (PSZ_AMD_DECODER_*)
DECODERS = (cz.DECODER_AUTO, cz.DECODER_LANE, cz.DECODER_WAVE)

CASES = [
    # (kind, dims, dtype, eb, zigzag, radius)
    ("smooth", (1000, 1, 1), np.float32, 1e-3, False, 512),
    ("smooth", (16384 * 3 + 11, 1, 1), np.float32, 1e-4, False, 512),
    ("walk", (200_003, 1, 1), np.float32, 1e-4, False, 512),
    ("smooth", (70, 45, 1), np.float32, 1e-3, False, 512),
    ("smooth", (3600, 1800, 1), np.float32, 1e-4, False, 512),
    ("smooth", (33, 17, 9), np.float32, 1e-3, False, 512),
    ("smooth", (64, 64, 64), np.float32, 1e-4, False, 512),
    ("smooth", (255, 257, 9), np.float32, 1e-4, False, 512),
    ("smooth", (100, 60, 40), np.float32, 1e-4, False, 512),
    ("smooth", (512, 256, 24), np.float32, 1e-4, False, 512),
    ("smooth", (130, 70, 30), np.float64, 1e-5, False, 512),
    ("smooth", (1000, 1, 1), np.float64, 1e-5, False, 512),
    ("smooth", (301, 77, 1), np.float64, 1e-5, False, 512),
    ("smooth", (64, 48, 40), np.float64, 1e-5, True, 512),
    ("smooth", (64, 64, 64), np.float32, 1e-4, True, 512),
    ("smooth", (5000, 1, 1), np.float32, 1e-4, True, 512),
    ("smooth", (300, 100, 1), np.float32, 1e-4, True, 512),
    ("smooth", (64, 40, 24), np.float32, 1e-3, False, 256),
    ("smooth", (64, 40, 24), np.float32, 1e-3, False, 64),
    ("int", (48, 40, 16), np.float32, 0.5, False, 512),
    ("noise", (40, 40, 40), np.float32, 1e-2, False, 512),
]


@pytest.mark.parametrize("kind,dims,dtype,eb,zigzag,radius", CASES,
                         ids=[f"{c[0]}-{'x'.join(map(str, c[1]))}-{np.dtype(c[2]).name}-{c[3]}-zz{int(c[4])}-r{c[5]}"
                              for c in CASES])
def test_parity_vs_oracle(oracle, kind, dims, dtype, eb, zigzag, radius):
    data = _field(kind, dims, dtype, seed=sum(dims))
    run_roundtrip(oracle, data, dims, eb, dtype, zigzag, radius)


EXACT_CASES = [c for c in CASES if c[1] in ((512, 256, 24), (3600, 1800, 1), (200_003, 1, 1), (130, 70, 30),
                                            (64, 64, 64))]


@pytest.mark.parametrize("kind,dims,dtype,eb,zigzag,radius", EXACT_CASES,
                         ids=[f"{c[0]}-{'x'.join(map(str, c[1]))}-{np.dtype(c[2]).name}-zz{int(c[4])}" for c in EXACT_CASES])
def test_parity_exact_reference_book(oracle, kind, dims, dtype, eb, zigzag, radius):
    """PSZ_AMD_CODEBOOK_EXACT: the reference's heap codebook of the full histogram, built on the
    host -- the Huffman segment equals the reference encoder's (byte for byte on the reference
    layout, chunk for chunk on the brick layout)."""
    data = _field(kind, dims, dtype, seed=sum(dims))
    run_roundtrip(oracle, data, dims, eb, dtype, zigzag, radius, codebook=cz.CODEBOOK_EXACT)


@pytest.mark.parametrize("sublen", [256, 1024, 4096])
def test_parity_sublen_override(oracle, sublen):
    dims = (64, 64, 32)
    data = datagen.smooth3d_np(dims, 5)
    arch, a = run_roundtrip(oracle, data, dims, 1e-4, sublen=sublen)
    assert a["sublen"] == sublen


@pytest.mark.parametrize("t,dims", [("t1", (256, 1, 1)), ("t2", (16, 16, 1)), ("t3", (8, 8, 8))])
def test_reference_kat_on_gpu(oracle, t, dims):
    """The reference's own KATs (correctness.inl) through the GPU path (eb=0.5)."""
    from conftest import GOLDEN

    k = np.load(os.path.join(GOLDEN, "kat_lorenzo.npz"))
    arch, a = run_roundtrip(oracle, k[f"{t}_in"], dims, 0.5)
    r = cz.Resource(cz.F4, dims)
    d_in = to_device(k[f"{t}_in"])
    r.compress(d_in.data_ptr(), 0.5)
    codes = d2h(r.internals().d_quant_codes, 2 * int(np.prod(dims)), np.uint16)
    np.testing.assert_array_equal(codes.astype(np.float32), k[f"{t}_comp_out"] + 512)


def test_single_symbol_and_constant_field(oracle):
    dims = (4096, 1, 1)
    data = np.full(4096, 0.0, np.float32)
    arch, a = run_roundtrip(oracle, data, dims, 1e-3)
    assert a["total_nbit"] == 4096  # 1-bit code per symbol (DESIGN.md deviation)


def test_decompress_with_fresh_manager_from_header(oracle):
    import torch

    dims = (96, 80, 40)
    data = datagen.smooth3d_np(dims, 9)
    r = cz.Resource(cz.F4, dims)
    d_in = to_device(data)
    ptr, nbytes, _ = r.compress(d_in.data_ptr(), 1e-4)
    arch = torch.from_numpy(d2h(ptr, nbytes).copy()).cuda()
    h = cz.psz_header.from_buffer_copy(arch[:176].cpu().numpy().tobytes())
    r2 = cz.Resource(None, None, header=h)
    out = empty_device(data.size, torch.float32)
    r2.decompress(arch.data_ptr(), nbytes, out.data_ptr())
    sync()
    assert np.max(np.abs(out.cpu().numpy().astype(np.float64) - data)) <= 1.001e-4


def test_manager_reuse_resets_state(oracle):
    """Appendix B.3: reusing a manager must not mix stale outliers/histogram."""
    dims = (64, 64, 16)
    r = cz.Resource(cz.F4, dims)
    d1 = to_device(datagen.smooth3d_np(dims, 1))
    d2 = to_device(datagen.smooth3d_np(dims, 2, noise=1e-2))
    r.compress(d1.data_ptr(), 1e-4)
    p2, n2, _ = r.compress(d2.data_ptr(), 1e-4)
    a2 = parse_archive(d2h(p2, n2).tobytes())
    codes, ov, oi = oracle.lorenzo_c(d2.cpu().numpy(), dims, 1e-4)
    assert a2["header"].splen == len(oi)
    np.testing.assert_array_equal(np.sort(a2["ol_idx"]), oi)


def test_outlier_capacity_grows_beyond_ten_percent(oracle):
    """Past the reference's 10 % outlier capacity (buf_comp.cc:87-88) the spill list grows and the
    call succeeds: nearly every element of uniform noise is an outlier, kept exactly."""
    dims = (200_000, 1, 1)
    data = np.random.default_rng(0).uniform(-1e3, 1e3, dims[0]).astype(np.float32)
    r = cz.Resource(cz.F4, dims)
    d_in = to_device(data)
    ptr, nbytes, st = r.compress(d_in.data_ptr(), 1e-4)
    assert st == cz.PSZ_SUCCESS
    a = parse_archive(d2h(ptr, nbytes).tobytes())
    codes, ov, oi = oracle.lorenzo_c(data, dims, 1e-4)
    assert a["header"].splen == len(oi) > dims[0] // 2
    np.testing.assert_array_equal(np.sort(a["ol_idx"]), oi)
    import torch

    out = torch.full(dims[:1], float("nan"), device="cuda")
    r.decompress(ptr, nbytes, out.data_ptr())
    sync()
    xg = out.cpu().numpy()
    np.testing.assert_array_equal(xg, oracle.lorenzo_x(codes, ov, oi, dims, 1e-4))
    # the capacity stays grown: a second call on the same manager succeeds directly
    ptr2, nb2, st2 = r.compress(d_in.data_ptr(), 1e-4)
    assert st2 == cz.PSZ_SUCCESS and nb2 == nbytes


def test_rel_mode(oracle):
    dims = (80, 60, 20)
    data = datagen.smooth3d_np(dims, 4) * 3.0 + 10.0
    r = cz.Resource(cz.F4, dims)
    d_in = to_device(data)
    ptr, nbytes, _ = r.compress(d_in.data_ptr(), 1e-4, cz.Rel)
    h = r.header
    rng = float(data.max()) - float(data.min())
    assert h.min_val == float(data.min()) and h.max_val == float(data.max())
    assert h.rc.eb == 1e-4 * rng and h.user_input_eb == 1e-4
    codes_o, _, _ = oracle.lorenzo_c(data, dims, 1e-4 * rng)
    np.testing.assert_array_equal(d2h(r.internals().d_quant_codes, 2 * data.size, np.uint16), codes_o)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("where", ["body", "body_end", "tail"])
def test_rel_mode_extrema_regions(dtype, where):
    """The extrema pass reads the field in 16-B groups (several per lane and iteration), then the
    last elements one by one: a minimum and maximum placed in the body, at the end of the grouped
    part and in the scalar tail must be found (extrema.cuhip.inl:86-208)."""
    dims = (307, 125, 121)  # n % 16 == 15: a ragged group count and a scalar tail for f32 and f64
    n = dims[0] * dims[1] * dims[2]
    e = 16 // np.dtype(dtype).itemsize
    groups = n // e
    assert groups % 4 and n % e
    data = (np.sin(np.arange(n) * 1e-3) * 5.0).astype(dtype)
    pos = {"body": (groups // 2) * e + 1, "body_end": (groups // 4 * 4) * e + 1, "tail": n - 1}[where]
    data[pos] = 40.0
    data[pos - 1] = -30.0
    r = cz.Resource(cz.F4 if dtype == np.float32 else cz.F8, dims)
    d_in = to_device(data)
    r.compress(d_in.data_ptr(), 1e-3, cz.Rel)
    h = r.header
    assert h.min_val == -30.0 and h.max_val == 40.0
    r.close()


@pytest.mark.parametrize("decoder", [cz.DECODER_WAVE, cz.DECODER_LANE, cz.DECODER_AUTO])
def test_long_chunks_high_entropy_all_decoders(oracle, decoder):
    """sublen 8192 with ~10-bit codes: the wave decoder's LDS staging would exceed its budget,
    so it stages what fits and reads the rest of a chunk from HBM."""
    n = 8192 * 6 + 77
    data = np.random.default_rng(12).random(n).astype(np.float32)
    r = cz.Resource(cz.F4, (n, 1, 1))
    r.set_sublen(8192)
    r.set_decoder(decoder)
    d_in = to_device(data)
    ptr, nbytes, _ = r.compress(d_in.data_ptr(), 1e-3)
    a = parse_archive(d2h(ptr, nbytes).tobytes())
    assert a["sublen"] == 8192 and a["total_nbit"] > 9 * n
    r.decode_codes(ptr)
    sync()
    codes_o, _, _ = oracle.lorenzo_c(data, (n, 1, 1), 1e-3)
    np.testing.assert_array_equal(d2h(r.internals().d_quant_codes, 2 * n, np.uint16), codes_o)
