"""Fused brick path (brick.hip): predictor+encoder and decoder+reconstructor in one pass each.

Parity is the same contract as the reference layout: quant codes (decoded back from the
archive with the general decoder), outlier set, histogram, codebook, par_nbit and every chunk's
cells equal the oracle's; the decompressed field equals the oracle's bit for bit.  Only chunk
placement differs (brick by brick, zero gaps), which par_entry records -- the reference decoder
reads chunk c at par_entry[c] (hf_kernels.cuhip.inl:386-391).
"""
import numpy as np
import pytest
import torch

import cusz_amd as cz
from cusz_amd import datagen
from gpu_util import d2h, empty_device, parse_archive, sync, to_device
from test_gpu_parity import run_roundtrip

pytestmark = pytest.mark.gpu

CASES = [
    # dims, dtype, eb, zigzag, radius, kind
    ((256, 8, 8), np.float32, 1e-4, False, 512, "smooth"),
    ((512, 64, 40), np.float32, 1e-4, False, 512, "smooth"),
    ((256, 13, 11), np.float32, 1e-3, False, 512, "smooth"),   # partial bricks in y and z
    ((768, 24, 17), np.float32, 1e-4, False, 512, "smooth"),   # 3 bricks along x, ragged z
    ((256, 40, 24), np.float64, 1e-5, False, 512, "smooth"),
    ((512, 16, 9), np.float64, 2e-5, False, 512, "smooth"),
    ((256, 32, 16), np.float32, 1e-4, True, 512, "smooth"),    # ZigZag
    ((256, 32, 16), np.float64, 1e-5, True, 512, "smooth"),
    ((256, 24, 16), np.float32, 1e-3, False, 64, "smooth"),    # small radius: many outliers
    ((256, 16, 16), np.float32, 1e-2, False, 512, "noise"),    # high entropy: HBM-read decode path,
    ((256, 16, 16), np.float32, 1e-2, True, 512, "noise"),     # and pass-1 byte codes escaping to u16
    ((256, 16, 16), np.float64, 3e-2, False, 256, "noise"),
    ((256, 16, 8), np.float32, 0.5, False, 512, "int"),
    # 1-D bricks: 64 chunks of 256; units of 64 tiles of 1024 in the decoder (ragged ends)
    ((16384, 1, 1), np.float32, 1e-4, False, 512, "smooth"),
    ((100_003, 1, 1), np.float32, 1e-4, False, 512, "hacc"),
    ((65536 * 3 + 1000, 1, 1), np.float32, 1e-3, False, 512, "hacc"),
    ((300, 1, 1), np.float32, 1e-4, False, 512, "smooth"),
    ((100_003, 1, 1), np.float64, 1e-4, False, 512, "hacc"),
    ((70_001, 1, 1), np.float32, 1e-4, True, 512, "hacc"),
    ((70_001, 1, 1), np.float64, 1e-4, True, 512, "hacc"),
    ((50_000, 1, 1), np.float32, 1e-2, False, 512, "noise"),
    ((50_000, 1, 1), np.float32, 1e-3, False, 64, "hacc"),     # many outliers per block row
    ((40_000, 1, 1), np.float32, 0.5, False, 512, "int"),
    # 2-D on linear bricks (x % 4 == 0, x >= 256): 2-D predictor, chunks as 1-D bricks place them
    ((3600, 90, 1), np.float32, 1e-4, False, 512, "cesm"),
    ((300, 97, 1), np.float32, 1e-4, False, 512, "cesm"),
    ((1024, 33, 1), np.float64, 1e-4, False, 512, "cesm"),
    ((3600, 40, 1), np.float32, 1e-4, True, 512, "cesm"),
    ((512, 64, 1), np.float32, 1e-2, False, 512, "noise"),
]


def _field(kind, dims, dtype, seed):
    n = int(np.prod(dims))
    rng = np.random.default_rng(seed)
    if kind == "smooth":
        return datagen.smooth3d_np(dims, seed, dtype=dtype)
    if kind == "noise":
        return rng.standard_normal(n).astype(dtype)
    if kind == "hacc":
        return datagen.hacc1d_np(n, seed).astype(dtype)
    if kind == "cesm":
        return datagen.cesm2d_np(dims[:2], seed).astype(dtype).reshape(-1)
    return np.cumsum(rng.integers(-3, 4, n)).astype(dtype)


@pytest.mark.parametrize("dims,dtype,eb,zz,radius,kind", CASES,
                         ids=[f"{'x'.join(map(str, c[0]))}-{np.dtype(c[1]).name}-{c[2]}-zz{int(c[3])}-r{c[4]}-{c[5]}"
                              for c in CASES])
def test_brick_parity(oracle, dims, dtype, eb, zz, radius, kind):
    data = _field(kind, dims, dtype, seed=sum(dims))
    # 2-D fields this small take the reference layout by default (too few bricks): force bricks
    layout = cz.LAYOUT_BRICK_FORCE if dims[1] > 1 and dims[2] == 1 else None
    arch, a = run_roundtrip(oracle, data, dims, eb, dtype, zz, radius, check_bound=kind != "noise", layout=layout)
    assert a["sublen"] == 256, "brick layout expected"


def test_brick_and_reference_layouts_decompress_identically(oracle):
    dims = (512, 48, 24)
    data = datagen.smooth3d_np(dims, 11)
    outs = []
    for layout in (cz.LAYOUT_BRICK, cz.LAYOUT_REFERENCE):
        arch, a = run_roundtrip(oracle, data, dims, 1e-4, layout=layout, codebook=cz.CODEBOOK_EXACT)
        outs.append(a)
    np.testing.assert_array_equal(np.sort(outs[0]["ol_idx"]), np.sort(outs[1]["ol_idx"]))
    np.testing.assert_array_equal(outs[0]["par_nbit"], outs[1]["par_nbit"])  # same chunking here


def test_reference_layout_archive_with_brick_sublen_uses_fused_decoder(oracle):
    """A reference-layout archive whose chunk length is the brick width (chunks in index order,
    not brick order) decodes through the fused decoder's per-chunk staging path."""
    dims = (256, 24, 16)
    data = datagen.smooth3d_np(dims, 3)
    run_roundtrip(oracle, data, dims, 1e-4, layout=cz.LAYOUT_REFERENCE, sublen=256)


def test_brick_rel_mode(oracle):
    dims = (256, 40, 20)
    data = datagen.smooth3d_np(dims, 4) * 3.0 + 10.0
    r = cz.Resource(cz.F4, dims)
    d_in = to_device(data)
    ptr, nbytes, _ = r.compress(d_in.data_ptr(), 1e-4, cz.Rel)
    assert r.internals().layout == cz.LAYOUT_BRICK
    rng = float(data.max()) - float(data.min())
    r.decode_codes(ptr)
    sync()
    codes_o, ov, oi = oracle.lorenzo_c(data, dims, 1e-4 * rng)
    np.testing.assert_array_equal(d2h(r.internals().d_quant_codes, 2 * data.size, np.uint16), codes_o)
    out = empty_device(data.size, torch.float32)
    r.decompress(ptr, nbytes, out.data_ptr())
    sync()
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.lorenzo_x(codes_o, ov, oi, dims, 1e-4 * rng))


def test_brick_repeat_is_deterministic():
    dims = (512, 64, 32)
    d_in = to_device(datagen.smooth3d_np(dims, 8))
    r = cz.Resource(cz.F4, dims)
    p1, n1, _ = r.compress(d_in.data_ptr(), 1e-4)
    a1 = d2h(p1, n1).tobytes()
    p2, n2, _ = r.compress(d_in.data_ptr(), 1e-4)
    assert d2h(p2, n2).tobytes() == a1
