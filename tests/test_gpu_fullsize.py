"""Full-size (BASELINE configs) checks through size-independent properties.

At 512^3 the CPU oracle would take minutes, so parity is established by
(a) tile independence: tile-aligned sub-blocks of the full field must produce exactly the
    oracle's codes/outliers for that sub-block alone (the reference predictor never reads
    across a tile, lrz_c.cuhip.inl:275-372), checked on several slabs;
(b) decode(encode(codes)) == codes, histogram == bincount(codes), #outliers == #(code==0);
(c) the error bound |x - x'| <= 1.001 eb on every element (compare.stl.inl:43-55).
"""
import numpy as np
import pytest
import torch

import cusz_amd as cz
from cusz_amd import datagen
from gpu_util import d2h, empty_device, parse_archive, sync

pytestmark = pytest.mark.gpu


def _check_full(oracle, d_in, dims, eb, slabs, dtype=np.float32):
    n = int(np.prod(dims))
    r = cz.Resource(cz.F4 if dtype == np.float32 else cz.F8, dims)
    ptr, nbytes, _ = r.compress(d_in.data_ptr(), eb)
    ino = r.internals()
    if ino.layout == cz.LAYOUT_BRICK:  # fused path: the codes exist only inside the archive
        r.decode_codes(ptr)
    codes_t = torch.empty(n, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    import ctypes as C
    from gpu_util import hip
    assert hip().hipMemcpy(C.c_void_p(codes_t.data_ptr()), C.c_void_p(ino.d_quant_codes), 2 * n, 3) == 0
    codes_i = codes_t.to(torch.int32) & 0xFFFF
    hist = torch.bincount(codes_i, minlength=1024).cpu().numpy()
    np.testing.assert_array_equal(d2h(ino.d_hist, 4096, np.uint32), hist)
    h = r.header
    assert h.splen == hist[0]
    # (a) tile independence vs the oracle on z-slabs
    x, y, z = dims
    host = d_in.cpu().numpy()
    codes_h = codes_i.cpu().numpy().astype(np.uint16)
    for z0, nz in slabs:
        sub = host[z0 * x * y:(z0 + nz) * x * y]
        c_o, _, _ = oracle.lorenzo_c(sub, (x, y, nz), eb)
        np.testing.assert_array_equal(codes_h[z0 * x * y:(z0 + nz) * x * y], c_o)
    # (b) decode(encode) idempotence through the archive, with both decoders
    for kind in (cz.DECODER_LANE, cz.DECODER_WAVE, cz.DECODER_AUTO):
        r.set_decoder(kind)
        codes_t.zero_()
        assert hip().hipMemcpy(C.c_void_p(ino.d_quant_codes), C.c_void_p(codes_t.data_ptr()), 2 * n, 3) == 0
        r.decode_codes(ptr)
        sync()
        dec = d2h(ino.d_quant_codes, 2 * n, np.uint16)
        np.testing.assert_array_equal(dec, codes_h, err_msg=f"decoder {kind}")
    # (c) error bound after a full decompress into a poisoned buffer
    out = empty_device(n, torch.float32 if dtype == np.float32 else torch.float64)
    out.fill_(float("nan"))
    r.decompress(ptr, nbytes, out.data_ptr())
    sync()
    err = (out.double() - d_in.double()).abs().max().item()
    assert err <= 1.001 * eb, err
    return nbytes


def test_config2_512cubed(oracle):
    dims = (512, 512, 512)
    d_in = datagen.smooth3d_torch(dims, seed=2)
    nbytes = _check_full(oracle, d_in, dims, 1e-4, slabs=[(0, 8), (256, 8), (504, 8)])
    assert nbytes < 512**3 * 4 / 3  # sanity: the field compresses


def test_config1_cesm_2d(oracle):
    dims = (3600, 1800, 1)
    host = datagen.cesm2d_np(dims[:2], seed=1)
    d_in = torch.from_numpy(host).cuda()
    r = cz.Resource(cz.F4, dims)
    ptr, nbytes, _ = r.compress(d_in.data_ptr(), 1e-4)
    if r.internals().layout == cz.LAYOUT_BRICK:  # the codes never reach HBM in index order
        r.decode_codes(ptr)
        sync()
    c_o, ov, oi = oracle.lorenzo_c(host, dims, 1e-4)
    np.testing.assert_array_equal(d2h(r.internals().d_quant_codes, 2 * host.size, np.uint16), c_o)
    out = empty_device(host.size, torch.float32)
    r.decompress(ptr, nbytes, out.data_ptr())
    sync()
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.lorenzo_x(c_o, ov, oi, dims, 1e-4))


def test_config3_hacc_1d_ragged(oracle):
    """N1 = 280,953,867 (N1 mod 1024 = 11 exercises the partial-tile path; Appendix B.1)."""
    n = 280_953_867
    g = torch.Generator(device="cuda")
    g.manual_seed(3)
    steps = torch.randn(n, generator=g, device="cuda", dtype=torch.float32) * 2e-3
    jump = torch.rand(n, generator=g, device="cuda") < 0.05
    steps = torch.where(jump, torch.rand(n, generator=g, device="cuda") * 256.0, steps)
    d_in = torch.remainder(torch.cumsum(steps.double(), 0), 256.0).float()
    del steps, jump
    r = cz.Resource(cz.F4, (n, 1, 1))
    ptr, nbytes, _ = r.compress(d_in.data_ptr(), 1e-4)
    h = r.header
    ino = r.internals()
    if ino.layout == cz.LAYOUT_BRICK:  # the codes never reach HBM in index order: decode them
        r.decode_codes(ptr)
        sync()
    # tail tile against the oracle (tile-independence), including the ragged last tile
    tail0 = (n // 1024 - 3) * 1024
    sub = d_in[tail0:].cpu().numpy()
    c_o, _, oi = oracle.lorenzo_c(sub, (sub.size, 1, 1), 1e-4)
    codes_tail = d2h(ino.d_quant_codes + 2 * tail0, 2 * sub.size, np.uint16)
    np.testing.assert_array_equal(codes_tail, c_o)
    a_cells = parse_archive(d2h(ptr, nbytes).tobytes())
    assert a_cells["ol_idx"].max() < n  # no spurious outliers past len (reference bug B.1)
    out = empty_device(n, torch.float32)
    r.decompress(ptr, nbytes, out.data_ptr())
    sync()
    err = (out.double() - d_in.double()).abs().max().item()
    assert err <= 1.001e-4 * 1.0 + 256 * 2**-23, err  # f32 prequant at |x|<256
