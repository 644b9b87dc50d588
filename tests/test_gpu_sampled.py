"""Sampled codebook (psz_amd_set_codebook: SAMPLED, the default, and STREAM): the codebook
comes from a sample plus one on every bin, built on the device (book_device.hh).  SAMPLED: pass 1
visits every 17th brick first (fewer bricks: 9th, 5th, 3rd, all) and a side-stream workgroup builds
the book from their histograms while pass 1 runs, then plan and pack as the exact mode.  STREAM:
k_brick3_sample takes a 1/16 sample of 32 x 8 x 8 units first, then one pass predicts and packs
(k_brick3_stream).

Parity contract: quant codes, outlier set and the decompressed field equal the oracle's (the
exact mode's) bit for bit; the Huffman segment equals the oracle encoder's output for the
oracle-computed sampled codebook (the same sample of the oracle's codes, the device book's
algorithm restated: orc_book_twoqueue_u2) -- revbook, par_nbit, every chunk's cells -- with the
chunks back to back (no gaps); the archive is an ordinary phf archive (the oracle's CPU decoder
reads it).
"""
import numpy as np
import pytest
import torch

import cusz_amd as cz
from cusz_amd import datagen
from gpu_util import chunk_cells, d2h, empty_device, expected_books, parse_archive, sync, to_device

pytestmark = pytest.mark.gpu


CASES = [
    # dims, dtype, eb, zigzag, radius, kind
    ((512, 64, 40), np.float32, 1e-4, False, 512, "smooth"),
    ((256, 13, 11), np.float32, 1e-3, False, 512, "smooth"),   # partial bricks in y and z
    ((768, 24, 17), np.float32, 1e-4, False, 512, "smooth"),
    ((256, 40, 24), np.float64, 1e-5, False, 512, "smooth"),
    ((256, 32, 16), np.float32, 1e-4, True, 512, "smooth"),    # ZigZag
    ((256, 24, 16), np.float32, 1e-3, False, 64, "smooth"),    # small radius: many outliers
    ((256, 16, 16), np.float32, 1e-2, False, 512, "noise"),    # u16 rows, long codes
    ((512, 16, 24), np.float32, 2e-3, False, 512, "noise"),    # ~10 bits/code: bricks outgrow the staging
    ((512, 128, 136), np.float32, 1e-4, False, 512, "smooth"),  # 1088 bricks: every 16th sampled
]


@pytest.mark.parametrize("mode", [cz.CODEBOOK_SAMPLED, cz.CODEBOOK_STREAM], ids=["sampled", "stream"])
@pytest.mark.parametrize("dims,dtype,eb,zz,radius,kind", CASES,
                         ids=[f"{'x'.join(map(str, c[0]))}-{np.dtype(c[1]).name}-{c[2]}-zz{int(c[3])}-r{c[4]}-{c[5]}"
                              for c in CASES])
def test_sampled_parity(oracle, dims, dtype, eb, zz, radius, kind, mode):
    n = int(np.prod(dims))
    if kind == "smooth":
        data = datagen.smooth3d_np(dims, sum(dims), dtype=dtype)
    else:
        data = np.random.default_rng(sum(dims)).standard_normal(n).astype(dtype)
    r = cz.Resource(cz.F4 if dtype == np.float32 else cz.F8, dims, cz.LorenzoZigZag if zz else cz.Lorenzo)
    r.set_codebook(mode)
    d_in = to_device(data)
    ptr, nbytes, _ = r.compress(d_in.data_ptr(), eb, cz.Abs, radius)
    arch = d2h(ptr, nbytes).tobytes()
    a = parse_archive(arch)
    h = a["header"]
    assert h.entry[5] == nbytes and a["sublen"] == 256
    ino = r.internals()
    assert ino.layout == cz.LAYOUT_BRICK

    codes_o, ov_o, oi_o = oracle.lorenzo_c(data, dims, eb, radius, zz)
    r.decode_codes(ptr)
    sync()
    codes_g = d2h(ino.d_quant_codes, 2 * n, np.uint16)
    mism = np.flatnonzero(codes_g != codes_o)
    assert mism.size == 0, f"{mism.size} code mismatches, first at {mism[:5]}"
    order = np.argsort(a["ol_idx"], kind="stable")
    np.testing.assert_array_equal(a["ol_idx"][order], oi_o)
    np.testing.assert_array_equal(a["ol_val"][order].view(np.uint32), ov_o.view(np.uint32))

    # Huffman segment: the oracle's encoding with the sampled codebook, chunks back to back
    bklen = 2 * radius
    book, rv = expected_books(oracle, r, codes_o, dims, bklen, ino.layout)
    nbit_o, entry_o, bs_o, tot_o = oracle.hf_encode(codes_o, book, 256)
    np.testing.assert_array_equal(a["revbook"], rv)
    np.testing.assert_array_equal(a["par_nbit"], nbit_o)
    ours, gaps = chunk_cells(a["par_nbit"], a["par_entry"], a["bitstream"])
    ref, _ = chunk_cells(nbit_o, entry_o, bs_o)
    np.testing.assert_array_equal(ours, ref)
    if mode == cz.CODEBOOK_STREAM:
        assert not gaps.any(), "the single pass leaves no gaps"
    else:
        assert not np.any(a["bitstream"][gaps]), "nonzero cells between brick regions"
    assert a["total_nbit"] == tot_o and a["total_ncell"] == a["bitstream"].size
    dec = oracle.hf_decode(a["bitstream"], a["revbook"], a["par_nbit"], a["par_entry"], 256, n, bklen)
    np.testing.assert_array_equal(dec, codes_o)

    xo = oracle.lorenzo_x(codes_o, ov_o, oi_o, dims, eb, radius, zz, dtype)
    out = empty_device(n, torch.float32 if dtype == np.float32 else torch.float64)
    out.fill_(float("nan"))
    r.decompress(ptr, nbytes, out.data_ptr())
    sync()
    ubits = np.uint64 if dtype == np.float64 else np.uint32
    bad = np.flatnonzero(out.cpu().numpy().view(ubits) != xo.view(ubits))
    assert bad.size == 0, f"{bad.size} reconstruction mismatches"
    r.close()


@pytest.mark.parametrize("mode", [cz.CODEBOOK_SAMPLED, cz.CODEBOOK_STREAM], ids=["sampled", "stream"])
def test_sampled_repeat_and_exact_switch(oracle, mode):
    """Repeated sampled compresses give the same bytes (the ticket and look-back state reset per
    call); switching back to EXACT gives the exact archive again; the field decompresses the same."""
    dims = (512, 64, 48)
    data = datagen.smooth3d_np(dims, 5)
    d_in = to_device(data)
    r = cz.Resource(cz.F4, dims)
    r.set_codebook(cz.CODEBOOK_EXACT)
    p0, n0, _ = r.compress(d_in.data_ptr(), 1e-4)
    exact = d2h(p0, n0).tobytes()
    r.set_codebook(mode)
    p1, n1, _ = r.compress(d_in.data_ptr(), 1e-4)
    s1 = d2h(p1, n1).tobytes()
    p2, n2, _ = r.compress(d_in.data_ptr(), 1e-4)
    assert d2h(p2, n2).tobytes() == s1
    outs = []
    for p, nb in ((p2, n2),):
        out = empty_device(data.size, torch.float32)
        r.decompress(p, nb, out.data_ptr())
        sync()
        outs.append(out.cpu().numpy())
    r.set_codebook(cz.CODEBOOK_EXACT)
    p3, n3, _ = r.compress(d_in.data_ptr(), 1e-4)
    assert d2h(p3, n3).tobytes() == exact
    out = empty_device(data.size, torch.float32)
    r.decompress(p3, n3, out.data_ptr())
    sync()
    np.testing.assert_array_equal(out.cpu().numpy(), outs[0])
    r.close()


@pytest.mark.parametrize("mode", [cz.CODEBOOK_SAMPLED, cz.CODEBOOK_STREAM], ids=["sampled", "stream"])
def test_sampled_full_size_config2(mode):
    """512^3 f32 (config 2): decompresses within eb; CR within 1 % of the exact mode's."""
    dims = (512, 512, 512)
    x = datagen.smooth3d_torch(dims, seed=2)
    r = cz.Resource(cz.F4, dims)
    r.set_codebook(cz.CODEBOOK_EXACT)
    _, n_exact, _ = r.compress(x.data_ptr(), 1e-4)
    r.set_codebook(mode)
    p, nb, _ = r.compress(x.data_ptr(), 1e-4)
    assert nb <= 1.01 * n_exact, (nb, n_exact)
    out = torch.empty_like(x)
    r.decompress(p, nb, out.data_ptr())
    torch.cuda.synchronize()
    assert float((out - x).abs().max()) <= 1.001e-4
    r.close()
