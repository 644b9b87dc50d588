"""Config 4 of BASELINE.json on one GPU: the six Nyx-like 512^3 f32 fields (datagen.nyx_fields_torch,
SURVEY.md §8d), each split into the 8 tile-aligned z-slabs of an 8-GPU run, one manager per slab
standing in for the ranks:
  value range per slab (psz_amd_value_range) -> the all-reduce's arithmetic (MAX of {-min, max})
  -> r2r 1e-4 bound; pass 1 per slab -> the histogram all-reduce's arithmetic (sum) -> finish per
  slab with the shared codebook -> psz_amd_merge_archives.
The merged archive must be byte-identical to one compress of the whole field, and decompress
within the bound.  The Rel-mode whole-field compress must arrive at the same bound."""
import numpy as np
import pytest
import torch

import cusz_amd as cz
from cusz_amd import datagen, shard
from gpu_util import d2h, sync

pytestmark = pytest.mark.gpu

FULL = (512, 512, 512)
WORLD = 8


@pytest.mark.parametrize("bound", ["r2r", "abs"])
def test_nyx_six_fields_sharded_equals_whole(bound):
    """r2r 1e-4 (the reference's runtests bound) and abs 1e-4 (SURVEY §8d's config-4 bound: the
    velocity fields are mostly outliers, far past the 10 % slots; the slots grow to the largest
    brick's count, so every cell stays in its brick's slot and the merge is still byte-exact)."""
    slabs = shard.plan_slabs(FULL, WORLD)
    assert [s.dims[2] for s in slabs] == [64] * WORLD
    st = torch.cuda.current_stream().cuda_stream
    res = [cz.Resource(cz.F4, s.dims, stream=st) for s in slabs]
    whole = cz.Resource(cz.F4, FULL, stream=st)
    for r in res + [whole]:  # the reference codebook on both sides (the single compress samples otherwise)
        r.set_codebook(cz.CODEBOOK_EXACT)
    out = torch.empty(FULL[0] * FULL[1] * FULL[2], dtype=torch.float32, device="cuda")
    hists = torch.zeros((WORLD, 1025), dtype=torch.int32, device="cuda")
    mm = torch.empty((WORLD, 2), dtype=torch.float64, device="cuda")
    r2r = 1e-4
    fields = datagen.nyx_fields_torch(FULL, device="cuda")
    assert len(fields) == 6
    for fi, f in enumerate(fields):
        views = [f[s.offset:s.offset + s.count] for s in slabs]
        for r, v, k in zip(res, views, range(WORLD)):
            r.value_range(v.data_ptr(), mm[k].data_ptr(), v.numel())
        sync()
        lo, hi = mm[:, 0].min().item(), mm[:, 1].max().item()
        assert lo == f.min().item() and hi == f.max().item()
        eb = r2r * (hi - lo) if bound == "r2r" else 1e-4
        for attempt in range(2):  # a slab past its slots: every slab repeats once (shard.py)
            for k, (r, v) in enumerate(zip(res, views)):
                r.compress_scan(v.data_ptr(), eb, hists[k].data_ptr())
            sync()
            g = hists.to(torch.int64).sum(0)
            assert int(g[:1024].sum().item()) == f.numel()
            assert attempt == 0 or int(g[1024].item()) == 0
            g32 = g.to(torch.int32).contiguous()
            parts, again = [], False
            for r in res:
                try:
                    ptr, nb, _ = r.compress_finish(g32.data_ptr())
                except cz.PszError as e:
                    assert e.status == cz.PSZ_WARN_OUTLIER_TOO_MANY and attempt == 0
                    again = True
                    continue
                parts.append(d2h(ptr, nb).tobytes())
            if not again:
                break
        assert len(parts) == WORLD
        merged = shard.merge(parts, FULL, [s.offset for s in slabs])
        ptr, nb, _ = whole.compress(f.data_ptr(), eb, cz.Abs)
        single = d2h(ptr, nb).tobytes()
        assert len(merged) == len(single), fi
        assert merged == single, f"field {fi}: merged archive differs from the whole-field archive"
        if bound == "r2r":  # Rel mode on the whole field finds the same absolute bound
            whole.compress(f.data_ptr(), r2r, cz.Rel)
            assert whole.header.rc.eb == eb
        # the merged archive decompresses within the bound
        d_arch = torch.frombuffer(bytearray(merged), dtype=torch.uint8).cuda()
        hdr = cz.psz_header.from_buffer_copy(merged[:176])
        rx = cz.Resource(cz.F4, FULL, stream=st, header=hdr)
        out.fill_(float("nan"))
        rx.decompress(d_arch.data_ptr(), len(merged), out.data_ptr())
        sync()
        err = (out.double() - f.double()).abs().max().item()
        ulp = 2.0 ** -23 * max(abs(lo), abs(hi))
        assert err <= 1.001 * eb + ulp, (fi, err, eb)
        rx.close()
        del d_arch
        fields[fi] = None  # free the field before the next one
    for r in res:
        r.close()
    whole.close()


def test_nyx_velocity_abs_1e4_beyond_outlier_cap(oracle):
    """SURVEY §8d's config-4 bound, abs 1e-4, on a Nyx-like velocity field (200 G): most elements
    are outliers, far past the reference's 10 % capacity (buf_comp.cc:87-88).  The capacity grows:
    on a tile-aligned slab the codes and outliers equal the oracle's and the field decompresses
    within the bound; the full 512 x 512 x 64 slab of an 8-rank run decompresses within it too."""
    small = (256, 64, 16)
    v = datagen.nyx_fields_torch((256, 64, 16), device="cuda")[1].contiguous()
    r = cz.Resource(cz.F4, small)
    ptr, nb, st = r.compress(v.data_ptr(), 1e-4)
    assert st == cz.PSZ_SUCCESS
    host = v.cpu().numpy()
    codes, ov, oi = oracle.lorenzo_c(host, small, 1e-4)
    assert r.header.splen == len(oi) > host.size // 10
    r.decode_codes(ptr)
    sync()
    got = d2h(r.internals().d_quant_codes, 2 * host.size, np.uint16)
    np.testing.assert_array_equal(got, codes)
    out = torch.empty(host.size, dtype=torch.float32, device="cuda")
    ptr, nb, st = r.compress(v.data_ptr(), 1e-4)
    r.decompress(ptr, nb, out.data_ptr())
    sync()
    np.testing.assert_array_equal(out.cpu().numpy(), oracle.lorenzo_x(codes, ov, oi, small, 1e-4))
    r.close()

    slab = (512, 512, 64)
    f = datagen.nyx_fields_torch(FULL, device="cuda", z0=0, z1=64)[1].contiguous()
    r = cz.Resource(cz.F4, slab)
    ptr, nb, st = r.compress(f.data_ptr(), 1e-4)
    assert st == cz.PSZ_SUCCESS and r.header.splen > f.numel() // 10
    out = torch.empty(f.numel(), dtype=torch.float32, device="cuda")
    r.decompress(ptr, nb, out.data_ptr())
    sync()
    err = (out.double() - f.double()).abs().max().item()
    assert err <= 1e-4 * 1.001 + 2.0 ** -23 * f.abs().max().item(), err
    r.close()
