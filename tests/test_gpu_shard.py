"""Sharded compress on the GPU, one process standing in for the ranks: every
slab is compressed by its own manager with pass 1 (psz_amd_compress_scan_*), the slab
histograms are summed (the all-reduce's arithmetic), every slab is finished with the shared
codebook (psz_amd_compress_finish), and psz_amd_merge_archives joins them.  The merged archive
must be byte-identical to the archive of one compress over the whole field, in both layouts,
and decompress to the same field."""
import numpy as np
import pytest
import torch

import cusz_amd as cz
from cusz_amd import datagen
from cusz_amd.shard import merge, plan_slabs
from gpu_util import d2h, parse_archive, sync, to_device

pytestmark = pytest.mark.gpu


def _whole(data, dims, eb, dtype, layout, sublen, codebook=cz.CODEBOOK_EXACT):
    r = cz.Resource(cz.F4 if dtype == np.float32 else cz.F8, dims)
    r.set_layout(layout)
    r.set_codebook(codebook)
    if sublen:
        r.set_sublen(sublen)
    ptr, nb, _ = r.compress(to_device(data).data_ptr(), eb)
    return d2h(ptr, nb).tobytes(), r


def _sharded(data, dims, world, eb, dtype, layout, sublen, codebook=cz.CODEBOOK_EXACT, hist_out=None):
    slabs = [s for s in plan_slabs(dims, world) if s.count]
    res, dins = [], []
    hists = torch.zeros((len(slabs), 1025), dtype=torch.int32, device="cuda")  # + the overflow word
    for i, s in enumerate(slabs):
        r = cz.Resource(cz.F4 if dtype == np.float32 else cz.F8, s.dims)
        r.set_layout(layout)
        r.set_codebook(codebook)
        if sublen:
            r.set_sublen(sublen)
        d = to_device(data[s.offset:s.offset + s.count])
        r.compress_scan(d.data_ptr(), eb, hists[i].data_ptr())
        res.append(r), dins.append(d)
    sync()
    g = hists.to(torch.int64).sum(0).to(torch.int32).contiguous()
    if hist_out is not None:
        hist_out.append(g[:1024].cpu().numpy().astype(np.uint32))
    parts = []
    for r in res:
        ptr, nb, _ = r.compress_finish(g.data_ptr())
        parts.append(d2h(ptr, nb).tobytes())
    return merge(parts, dims, [s.offset for s in slabs])


@pytest.mark.parametrize("dims,world,dtype,layout,sublen", [
    ((256, 32, 40), 2, np.float32, cz.LAYOUT_BRICK, 0),
    ((256, 32, 40), 3, np.float32, cz.LAYOUT_BRICK, 0),
    ((512, 24, 64), 4, np.float32, cz.LAYOUT_BRICK, 0),
    ((256, 16, 24), 3, np.float64, cz.LAYOUT_BRICK, 0),
    ((256, 32, 40), 3, np.float32, cz.LAYOUT_REFERENCE, 256),
    ((96, 40, 48), 2, np.float32, cz.LAYOUT_REFERENCE, 768),
])
def test_sharded_merge_equals_whole_field(dims, world, dtype, layout, sublen):
    data = datagen.smooth3d_np(dims, 31, dtype=dtype)
    eb = 1e-4
    single, r = _whole(data, dims, eb, dtype, layout, sublen)
    merged = _sharded(data, dims, world, eb, dtype, layout, sublen)
    assert len(merged) == len(single)
    assert merged == single
    # the merged archive decompresses through the ordinary API
    d_arch = torch.frombuffer(bytearray(merged), dtype=torch.uint8).cuda()
    out = torch.full((data.size,), float("nan"), dtype=torch.float32 if dtype == np.float32 else torch.float64,
                     device="cuda")
    r.decompress(d_arch.data_ptr(), len(merged), out.data_ptr())
    sync()
    err = np.abs(out.cpu().numpy().astype(np.float64) - data.astype(np.float64)).max()
    assert err <= 1.001 * eb


@pytest.mark.parametrize("dims,world,layout", [((256, 32, 40), 3, cz.LAYOUT_BRICK),
                                               ((256, 32, 40), 3, cz.LAYOUT_REFERENCE),
                                               ((100_000, 1, 1), 2, cz.LAYOUT_BRICK)])
def test_sharded_device_book(oracle, dims, world, layout):
    """The default codebook mode on the sharded path: every rank builds the same device book from
    the reduced histogram (no host round trip): the merged archive's reverse book is the oracle's
    two-queue book of that histogram, and it decompresses within the bound."""
    x, y, z = dims
    data = (datagen.smooth3d_np(dims, 5) if z > 1 else datagen.hacc1d_np(x, 5)).astype(np.float32)
    eb = 1e-4
    hist = []
    merged = _sharded(data, dims, world, eb, np.float32, layout, 0, codebook=cz.CODEBOOK_SAMPLED, hist_out=hist)
    _, rv = oracle.book_twoqueue(hist[0], 1024, smooth=0)
    np.testing.assert_array_equal(parse_archive(merged)["revbook"], rv)
    d_arch = torch.frombuffer(bytearray(merged), dtype=torch.uint8).cuda()
    out = torch.full((data.size,), float("nan"), dtype=torch.float32, device="cuda")
    rx = cz.Resource(cz.F4, dims, header=cz.psz_header.from_buffer_copy(merged[:176]))
    rx.decompress(d_arch.data_ptr(), len(merged), out.data_ptr())
    sync()
    err = np.abs(out.cpu().numpy().astype(np.float64) - data.astype(np.float64)).max()
    assert err <= 1.001 * eb + 2.0 ** -23 * float(np.abs(data).max())


@pytest.mark.parametrize("dims,world", [((256, 32, 40), 3), ((512, 24, 64), 4)])
def test_sharded_default_mode_decodes_like_whole_field(dims, world):
    """Default (SAMPLED) mode: the whole-field compress takes a sampled host book and the sharded
    finish a device book of the reduced histogram, so the archives differ; the quantization codes
    and outliers do not, so both decompress to the IDENTICAL field, within the bound, and the
    sizes stay within 1 %."""
    data = datagen.smooth3d_np(dims, 17)
    eb = 1e-4
    single, r = _whole(data, dims, eb, np.float32, cz.LAYOUT_BRICK, 0, codebook=cz.CODEBOOK_SAMPLED)
    merged = _sharded(data, dims, world, eb, np.float32, cz.LAYOUT_BRICK, 0, codebook=cz.CODEBOOK_SAMPLED)
    assert abs(len(merged) - len(single)) <= 0.01 * len(single)
    outs = []
    for arch in (single, merged):
        d_arch = torch.frombuffer(bytearray(arch), dtype=torch.uint8).cuda()
        out = torch.full((data.size,), float("nan"), dtype=torch.float32, device="cuda")
        rx = cz.Resource(cz.F4, dims, header=cz.psz_header.from_buffer_copy(arch[:176]))
        rx.decompress(d_arch.data_ptr(), len(arch), out.data_ptr())
        sync()
        outs.append(out.cpu().numpy())
    np.testing.assert_array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))
    assert np.abs(outs[0].astype(np.float64) - data.astype(np.float64)).max() <= 1.001 * eb


def test_scan_then_finish_equals_compress():
    dims = (256, 24, 16)
    data = datagen.smooth3d_np(dims, 7)
    single, _ = _whole(data, dims, 1e-4, np.float32, cz.LAYOUT_BRICK, 0)
    r = cz.Resource(cz.F4, dims)
    r.set_codebook(cz.CODEBOOK_EXACT)
    d = to_device(data)
    h = torch.zeros(1025, dtype=torch.int32, device="cuda")
    r.compress_scan(d.data_ptr(), 1e-4, h.data_ptr())
    ptr, nb, _ = r.compress_finish(0)  # the slab's own histogram
    assert d2h(ptr, nb).tobytes() == single
    sync()
    assert int(h[:1024].sum().item()) == data.size and int(h[1024].item()) == 0  # counts, no overflow


def test_analyze_exports_histogram(oracle):
    dims = (96, 64, 24)
    data = datagen.smooth3d_np(dims, 2)
    r = cz.Resource(cz.F4, dims)
    d = to_device(data)
    hist = np.zeros(1024, np.uint32)
    st = cz.lib().psz_compress_analyize_float(r._h, cz.psz_rc2(cz.Abs, 1e-4, 512), cz.C.c_void_p(d.data_ptr()),
                                              hist.ctypes.data_as(cz.C.c_void_p))
    assert st == cz.PSZ_SUCCESS
    codes, _, _ = oracle.lorenzo_c(data, dims, 1e-4)
    np.testing.assert_array_equal(hist, oracle.histogram(codes))


def test_sharded_outlier_overflow_repeats_together():
    """One slab past its outlier capacity (uniform noise), the other well within it: the summed
    overflow word makes BOTH finishes warn, the overflowing slab's capacity grows, and the
    repeated step gives archives that merge into the whole field's archive (error-bounded)."""
    dims = (131072, 1, 1)
    rng = np.random.default_rng(11)
    h = dims[0] // 2
    data = np.concatenate([np.cumsum(rng.normal(0, 1e-5, h)), rng.uniform(-1e3, 1e3, h)]).astype(np.float32)
    slabs = plan_slabs(dims, 2)
    res = [cz.Resource(cz.F4, s.dims) for s in slabs]
    dins = [to_device(data[s.offset:s.offset + s.count]) for s in slabs]
    hists = torch.zeros((2, 1025), dtype=torch.int32, device="cuda")
    for attempt in range(2):
        for i, r in enumerate(res):
            r.compress_scan(dins[i].data_ptr(), 1e-4, hists[i].data_ptr())
        sync()
        g = hists.to(torch.int64).sum(0).to(torch.int32).contiguous()
        if attempt == 0:
            assert int(g[1024].item()) > 0  # slab 1 overflowed
        sts, parts = [], []
        for r in res:
            try:
                ptr, nb, _ = r.compress_finish(g.data_ptr())
                parts.append(d2h(ptr, nb).tobytes())
                sts.append(cz.PSZ_SUCCESS)
            except cz.PszError as e:
                sts.append(e.status)
        if attempt == 0:
            assert sts == [cz.PSZ_WARN_OUTLIER_TOO_MANY] * 2
    assert sts == [cz.PSZ_SUCCESS] * 2
    merged = cz.merge_archives(parts, dims, [s.offset for s in slabs])
    hdr = cz.psz_header.from_buffer_copy(merged[:176])
    rf = cz.Resource(cz.F4, dims, header=hdr)
    d_arch = torch.frombuffer(bytearray(merged), dtype=torch.uint8).to("cuda")
    out = torch.empty(dims[0], dtype=torch.float32, device="cuda")
    rf.decompress(d_arch.data_ptr(), len(merged), out.data_ptr())
    sync()
    # f32 reconstruction at |x| ~ 1e3: its rounding adds to the bound (as bench.py's check)
    assert np.abs(out.cpu().numpy().astype(np.float64) - data).max() <= 1.001e-4 + 2.0 ** -23 * np.abs(data).max()
