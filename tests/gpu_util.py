"""Device-memory helpers for the GPU tests (torch for allocation, hip runtime for copies)."""
import ctypes as C

import numpy as np
import torch  # noqa: F401  (before any HIP runtime is loaded: see cusz_amd.lib)

import cusz_amd as cz

_hip = None


def hip():
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipMemcpy.restype = C.c_int
        _hip.hipDeviceSynchronize.restype = C.c_int
    return _hip


D2H, H2D, D2D = 2, 1, 3


def d2h(ptr: int, nbytes: int, dtype=np.uint8) -> np.ndarray:
    out = np.empty(nbytes, np.uint8)
    if nbytes:
        st = hip().hipMemcpy(out.ctypes.data_as(C.c_void_p), C.c_void_p(ptr), nbytes, D2H)
        assert st == 0, st
    return out.view(dtype)


def to_device(a: np.ndarray):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def empty_device(n: int, dtype):
    import torch

    return torch.empty(n, dtype=dtype, device="cuda")


def sync():
    import torch

    torch.cuda.synchronize()


def parse_archive(arch: bytes, bklen=1024):
    """Split a cuSZ archive into its segments (header.h:19-48, hf.h:40-46)."""
    import struct

    import cusz_amd

    h = cusz_amd.psz_header.from_buffer_copy(arch[:176])
    phf = arch[h.entry[2]:h.entry[3]]
    bklen_, sublen, pardeg = struct.unpack_from("<iii", phf, 0)
    bklen_ &= 0xFFFF
    orig, tnbit, tncell = struct.unpack_from("<QQQ", phf, 16)
    pent = struct.unpack_from("<6I", phf, 40)
    rvbk = np.frombuffer(phf[pent[1]:pent[2]], np.uint8)
    par_nbit = np.frombuffer(phf[pent[2]:pent[3]], np.uint32)
    par_entry = np.frombuffer(phf[pent[3]:pent[4]], np.uint32)
    bitstream = np.frombuffer(phf[pent[4]:pent[5]], np.uint32)
    cells = np.frombuffer(arch[h.entry[3]:h.entry[4]], np.uint32).reshape(-1, 2)
    return dict(header=h, phf=phf, bklen=bklen_, sublen=sublen, pardeg=pardeg, original_len=orig,
                total_nbit=tnbit, total_ncell=tncell, phf_entry=pent, revbook=rvbk, par_nbit=par_nbit,
                par_entry=par_entry, bitstream=bitstream, ol_val=cells[:, 0].view(np.float32).copy(),
                ol_idx=cells[:, 1].copy())


def chunk_cells(par_nbit, par_entry, bitstream):
    """Concatenate every chunk's cells in chunk order (chunk c: ceil(nbit/32) cells at par_entry[c]),
    so archives with different chunk placement compare cell for cell.  Also returns the mask of
    bitstream cells no chunk covers (the brick layout's gaps)."""
    nc = ((par_nbit.astype(np.int64) + 31) >> 5)
    starts = par_entry.astype(np.int64)
    tot = int(nc.sum())
    idx = np.repeat(starts - np.concatenate(([0], np.cumsum(nc)[:-1])), nc) + np.arange(tot)
    covered = np.zeros(bitstream.size, bool)
    covered[idx] = True
    return bitstream[idx], ~covered


def expected_books(oracle, r, codes, dims, bklen, layout, spline=False):
    """The codebook a compress used (psz_amd_set_codebook): EXACT -> the reference's heap book of
    the full histogram; SAMPLED (default) -> on 3-D and 1-D bricks the two-queue book (restated by
    orc_book_twoqueue_u2) of pass 1's brick sample + 1 per bin (built on the host mid-pass), for
    spline the two-queue book of the full histogram (device), elsewhere the exact book;
    STREAM -> the device book of the 32 x 8 x 8-unit sample + 1 on 3-D bricks."""
    if r.codebook == cz.CODEBOOK_EXACT:
        return oracle.codebook(oracle.histogram(codes, bklen), bklen)
    x, y, z = (tuple(dims) + (1, 1))[:3]
    if r.codebook == cz.CODEBOOK_STREAM and layout == cz.LAYOUT_BRICK and z > 1:
        return oracle.book_twoqueue(oracle.sample_histogram(codes, (x, y, z), bklen, "units"), bklen, smooth=1)
    if layout == cz.LAYOUT_BRICK and (z > 1 or y == 1):  # 3-D and 1-D bricks sample inside pass 1
        # the two-queue book of sample + 1, built on the host while pass 1 goes on
        return oracle.book_twoqueue(oracle.sample_histogram(codes, (x, y, z), bklen), bklen, smooth=1)
    if spline:
        return oracle.book_twoqueue(oracle.histogram(codes, bklen), bklen, smooth=0)
    return oracle.codebook(oracle.histogram(codes, bklen), bklen)


def check_phf_against_oracle(a, info, seg_o, layout):
    """Huffman segment parity.  Reference layout: byte-identical.  Brick layout: identical
    revbook and par_nbit, every chunk's cells identical, the gaps between brick regions zero."""
    np.testing.assert_array_equal(a["revbook"], info["revbook"])
    np.testing.assert_array_equal(a["par_nbit"], info["par_nbit"])
    if layout == 1:
        np.testing.assert_array_equal(a["par_entry"], info["par_entry"])
        np.testing.assert_array_equal(a["bitstream"], info["bitstream"])
        assert a["phf"] == seg_o, "phf segment bytes differ"
        return
    ours, gaps = chunk_cells(a["par_nbit"], a["par_entry"], a["bitstream"])
    ref, _ = chunk_cells(info["par_nbit"], info["par_entry"], info["bitstream"])
    np.testing.assert_array_equal(ours, ref)
    assert not np.any(a["bitstream"][gaps]), "nonzero cells between brick regions"
    assert a["total_nbit"] == int(info["par_nbit"].astype(np.int64).sum())
    assert a["total_ncell"] == a["bitstream"].size
