"""oracle/pyoracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes bindings for the CPU oracle (liboracle.so, the clean-room restatement in
psz_oracle.c) and, when it has been built, for the compiled reference CPU path
(_ref/libpszref.so, see Makefile target `ref`).  Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg import this module, and only as a checker / baseline;
the product path (cusz_amd/) never does.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libpszref.so")

_P = C.c_void_p
_SZ = C.c_size_t


def build(ref: bool = True) -> None:
    """Compile liboracle.so (and _ref/libpszref.so when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE, "liboracle.so"], check=True)
    if ref and os.path.isdir(os.environ.get("PSZ_REFERENCE", "/root/reference")):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build(ref=False)
        L = C.CDLL(LIB_PATH)
        for name in ("orc_lorenzo_c_f32", "orc_lorenzo_c_f64"):
            f = getattr(L, name)
            f.restype = _SZ
            f.argtypes = [_P, _SZ, _SZ, _SZ, C.c_double, C.c_uint16, C.c_int, _P, _P, _P, _SZ]
        for name in ("orc_lorenzo_x_f32", "orc_lorenzo_x_f64"):
            f = getattr(L, name)
            f.restype = None
            f.argtypes = [_P, _P, _P, _SZ, _SZ, _SZ, _SZ, C.c_double, C.c_uint16, C.c_int, _P]
        for name in ("orc_spline3_c_f32", "orc_spline3_c_f64"):
            f = getattr(L, name)
            f.restype = _SZ
            f.argtypes = [_P, _SZ, _SZ, _SZ, C.c_double, C.c_int, _P, _P, _P, _P, _SZ]
        for name in ("orc_spline3_x_f32", "orc_spline3_x_f64"):
            f = getattr(L, name)
            f.restype = None
            f.argtypes = [_P, _P, _P, _P, _SZ, _SZ, _SZ, _SZ, C.c_double, C.c_int, _P]
        L.orc_histogram_u2.argtypes = [_P, _SZ, _P, C.c_int]
        L.orc_build_codebook_u2.restype = C.c_int
        L.orc_build_codebook_u2.argtypes = [_P, C.c_int, _P, _P]
        L.orc_huffman_lengths.restype = C.c_int
        L.orc_huffman_lengths.argtypes = [_P, C.c_int, _P]
        L.orc_book_twoqueue_u2.restype = C.c_int
        L.orc_book_twoqueue_u2.argtypes = [_P, C.c_int, C.c_uint32, _P, _P]
        L.orc_coarse_tune.argtypes = [_SZ, C.c_int, C.c_int, _P, _P]
        L.orc_hf_encode_u2.restype = _SZ
        L.orc_hf_encode_u2.argtypes = [_P, _SZ, _P, C.c_int, _P, _P, _P, _SZ, _P]
        L.orc_hf_decode_u2.argtypes = [_P, _P, C.c_int, _P, _P, C.c_int, C.c_int, _SZ, _P]
        _lib = L
    return _lib


def ref_available() -> bool:
    return os.path.exists(REF_PATH)


def ref():
    global _ref
    if _ref is None:
        R = C.CDLL(REF_PATH)
        R.ref_c_lorenzo_f32.restype = C.c_uint32
        R.ref_c_lorenzo_f32.argtypes = [_P, _SZ, _SZ, _SZ, C.c_double, C.c_uint16, _P, _P, _P, _SZ]
        R.ref_x_lorenzo_f32.argtypes = [_P, _P, _P, _SZ, _SZ, _SZ, C.c_double, C.c_uint16]
        for fn in (R.ref_c_lorenzo_zz_f32, R.ref_c_lorenzo3d_f64):
            fn.restype = C.c_uint32
            fn.argtypes = [_P, _SZ, _SZ, _SZ, C.c_double, C.c_uint16, _P, _P, _P, _SZ]
        R.ref_scatter_f32.argtypes = [_P, _P, C.c_uint32, _P]
        R.ref_histogram_u2.argtypes = [_P, _SZ, _P, C.c_uint16]
        R.ref_build_codebook_u2.restype = C.c_int
        R.ref_build_codebook_u2.argtypes = [_P, C.c_int, _P, _P]
        R.ref_time_stages_f32.argtypes = [_P, _SZ, _SZ, _SZ, C.c_double, C.c_uint16, _P]
        R.ref_time_stages_par_f32.argtypes = [_P, C.c_int, _P, _P, C.c_double, C.c_uint16, _P]
        R.ref_time_stages_par_f32.restype = C.c_double
        _ref = R
    return _ref


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_P)


# --------------------------------------------------------------------------- oracle
def lorenzo_c(data: np.ndarray, dims, eb: float, radius: int = 512, zigzag: bool = False):
    """-> (codes u16[N], ol_val f32[k], ol_idx u32[k]) with outliers sorted by index."""
    data = np.ascontiguousarray(data)
    x, y, z = dims
    n = x * y * z
    assert data.size == n
    codes = np.zeros(n, np.uint16)
    cap = n
    ov = np.zeros(max(cap, 1), np.float32)
    oi = np.zeros(max(cap, 1), np.uint32)
    f = lib().orc_lorenzo_c_f64 if data.dtype == np.float64 else lib().orc_lorenzo_c_f32
    assert data.dtype in (np.float32, np.float64)
    k = f(_ptr(data), x, y, z, eb, radius, int(zigzag), _ptr(codes), _ptr(ov), _ptr(oi), cap)
    return codes, ov[:k].copy(), oi[:k].copy()


def lorenzo_x(codes, ol_val, ol_idx, dims, eb, radius=512, zigzag=False, dtype=np.float32):
    x, y, z = dims
    n = x * y * z
    codes = np.ascontiguousarray(codes, np.uint16)
    ol_val = np.ascontiguousarray(ol_val, np.float32)
    ol_idx = np.ascontiguousarray(ol_idx, np.uint32)
    out = np.zeros(n, dtype)
    f = lib().orc_lorenzo_x_f64 if dtype == np.float64 else lib().orc_lorenzo_x_f32
    f(_ptr(codes), _ptr(ol_val), _ptr(ol_idx), len(ol_idx), x, y, z, eb, radius, int(zigzag), _ptr(out))
    return out


def spline_anchor_len(dims):
    x, y, z = dims
    return ((x + 7) // 8) * ((y + 7) // 8) * ((z + 7) // 8)


def spline3_c(data: np.ndarray, dims, eb: float, radius: int = 512):
    """cuSZ-i spline3 (parity unpinned) -> (codes u16[N], anchors T[A], ol_val f32[k], ol_idx u32[k]);
    outliers in tile order, then (z,y,x) inside the 32x8x8 tile."""
    data = np.ascontiguousarray(data)
    x, y, z = dims
    n = x * y * z
    assert data.size == n and data.dtype in (np.float32, np.float64)
    codes = np.zeros(n, np.uint16)
    anchors = np.zeros(spline_anchor_len(dims), data.dtype)
    ov = np.zeros(max(n, 1), np.float32)
    oi = np.zeros(max(n, 1), np.uint32)
    f = lib().orc_spline3_c_f64 if data.dtype == np.float64 else lib().orc_spline3_c_f32
    k = f(_ptr(data), x, y, z, eb, radius, _ptr(codes), _ptr(anchors), _ptr(ov), _ptr(oi), n)
    return codes, anchors, ov[:k].copy(), oi[:k].copy()


def spline3_x(codes, anchors, ol_val, ol_idx, dims, eb, radius=512):
    x, y, z = dims
    n = x * y * z
    anchors = np.ascontiguousarray(anchors)
    codes = np.ascontiguousarray(codes, np.uint16)
    ol_val = np.ascontiguousarray(ol_val, np.float32)
    ol_idx = np.ascontiguousarray(ol_idx, np.uint32)
    out = np.zeros(n, anchors.dtype)
    f = lib().orc_spline3_x_f64 if anchors.dtype == np.float64 else lib().orc_spline3_x_f32
    f(_ptr(codes), _ptr(anchors), _ptr(ol_val), _ptr(ol_idx), len(ol_idx), x, y, z, eb, radius, _ptr(out))
    return out


def histogram(codes, bklen=1024):
    codes = np.ascontiguousarray(codes, np.uint16)
    h = np.zeros(bklen, np.uint32)
    lib().orc_histogram_u2(_ptr(codes), codes.size, _ptr(h), bklen)
    return h


def codebook(hist, bklen=1024):
    hist = np.ascontiguousarray(hist, np.uint32)
    book = np.zeros(bklen, np.uint32)
    rv = np.zeros(4 * 64 + 2 * bklen, np.uint8)
    nb = lib().orc_build_codebook_u2(_ptr(hist), bklen, _ptr(book), _ptr(rv))
    assert nb == rv.size
    return book, rv


def book_twoqueue(hist, bklen=1024, smooth=0):
    """The device codebook's algorithm (book_device.hh) restated: two-queue Huffman over
    (weight, symbol)-sorted leaves of hist + smooth, reference canonisation -> (book, revbook)."""
    hist = np.ascontiguousarray(hist, np.uint32)
    book = np.zeros(bklen, np.uint32)
    rv = np.zeros(4 * 64 + 2 * bklen, np.uint8)
    nb = lib().orc_book_twoqueue_u2(_ptr(hist), bklen, smooth, _ptr(book), _ptr(rv))
    assert nb == rv.size
    return book, rv


def sample_bricks(nbricks):
    """The codebook sample inside pass 1 (cusz_amd/csrc/brick.hip brick_sample_plan): bricks
    j * stride + stride // 2 with stride 33 / 17 / 9 / 5 / 3 from 8192 / 4352 / 2304 / 1280 / 768
    bricks up, else every brick."""
    stride = (33 if nbricks >= 8192 else 17 if nbricks >= 4352 else 9 if nbricks >= 2304 else 5 if nbricks >= 1280
              else 3 if nbricks >= 768 else 1)
    if stride == 1:
        return np.arange(nbricks)
    b = np.arange(0, nbricks, stride) + stride // 2
    return b[b < nbricks]


def sample_histogram(codes, dims, bklen=1024, scheme="bricks"):
    """The sampled codebook's histogram.
    scheme "bricks" (PSZ_AMD_CODEBOOK_SAMPLED, brick layout): the codes of the sample bricks
      (sample_bricks); a 3-D brick is 256 x 8 x 8 elements, index (bz * nby + by) * nbx + bx, a
      1-D brick 16384 consecutive elements.
    scheme "units" (PSZ_AMD_CODEBOOK_STREAM, k_brick3_sample): units of 32 x 8 x 8 elements (four
      8^3 Lorenzo tiles), unit u = (uz * nuy + uy) * nux + ux; from 4096 units up every 16th unit,
      u = 16 i + i % 16 (cycling through the x positions), else every unit.
    Only in-field elements count."""
    x, y, z = dims
    h = np.zeros(bklen, np.int64)
    if scheme == "bricks":
        if y == 1 and z == 1:
            c = np.asarray(codes).reshape(-1)
            for b in sample_bricks((x + 16383) // 16384):
                h += np.bincount(c[b * 16384:(b + 1) * 16384], minlength=bklen)[:bklen]
            return h.astype(np.uint32)
        nbx, nby, nbz = x // 256, (y + 7) // 8, (z + 7) // 8
        c = np.asarray(codes).reshape(z, y, x)
        for b in sample_bricks(nbx * nby * nbz):
            bx, t = b % nbx, b // nbx
            by, bz = t % nby, t // nby
            blk = c[bz * 8:bz * 8 + 8, by * 8:by * 8 + 8, bx * 256:bx * 256 + 256]
            h += np.bincount(blk.reshape(-1), minlength=bklen)[:bklen]
        return h.astype(np.uint32)
    nux, nuy, nuz = x // 32, (y + 7) // 8, (z + 7) // 8
    units = nux * nuy * nuz
    stride = 16 if units >= 256 * 16 else 1
    c = np.asarray(codes).reshape(z, y, x)
    for i in range((units + stride - 1) // stride):
        u = i * stride + i % stride
        if u >= units:
            continue
        ux, t = u % nux, u // nux
        uy, uz = t % nuy, t // nuy
        blk = c[uz * 8:uz * 8 + 8, uy * 8:uy * 8 + 8, ux * 32:ux * 32 + 32]
        h += np.bincount(blk.reshape(-1), minlength=bklen)[:bklen]
    return h.astype(np.uint32)


def huffman_lengths(hist, bklen=1024):
    hist = np.ascontiguousarray(hist, np.uint32)
    lens = np.zeros(bklen, np.uint8)
    lib().orc_huffman_lengths(_ptr(hist), bklen, _ptr(lens))
    return lens


def coarse_tune(n, n_cu=256, max_threads=1024):
    s = C.c_int()
    p = C.c_int()
    lib().orc_coarse_tune(n, n_cu, max_threads, C.byref(s), C.byref(p))
    return s.value, p.value


def hf_encode(codes, book, sublen):
    codes = np.ascontiguousarray(codes, np.uint16)
    n = codes.size
    pardeg = (n - 1) // sublen + 1
    nbit = np.zeros(pardeg, np.uint32)
    entry = np.zeros(pardeg, np.uint32)
    cap = n  # <= 27 bits per symbol -> worst case n cells
    bs = np.zeros(cap + 1, np.uint32)
    tot = C.c_uint64()
    ncell = lib().orc_hf_encode_u2(_ptr(codes), n, _ptr(book), sublen, _ptr(nbit), _ptr(entry),
                                   _ptr(bs), cap, C.byref(tot))
    assert ncell != 2**64 - 1
    return nbit, entry, bs[:ncell].copy(), tot.value


def hf_decode(bitstream, revbook, par_nbit, par_entry, sublen, n, bklen=1024):
    out = np.zeros(n, np.uint16)
    bs = np.ascontiguousarray(np.concatenate([bitstream, np.zeros(1, np.uint32)]), np.uint32)
    lib().orc_hf_decode_u2(_ptr(bs), _ptr(np.ascontiguousarray(revbook, np.uint8)), bklen,
                           _ptr(np.ascontiguousarray(par_nbit, np.uint32)),
                           _ptr(np.ascontiguousarray(par_entry, np.uint32)), sublen,
                           len(par_nbit), n, _ptr(out))
    return out


# ---------------------------------------------------------------- archive (restated)
PSZ_HEADER_BYTES = 176  # psz/include/cusz/header.h:19-48
PHF_HEADER_BYTES = 64   # codec/hf/include/hf.h:40-46
PHF_FORCED_ALIGN = 128  # hf.h:28


def phf_header_bytes(bklen, sublen, pardeg, original_len, total_nbit, total_ncell, entry):
    """phf_header layout: int bklen:16 @0, sublen @4, pardeg @8, original_len @16,
    total_nbit @24, total_ncell @32, entry u32[6] @40 (64 B)."""
    b = struct.pack("<iii4xQQQ6I", bklen & 0xFFFF, sublen, pardeg, original_len, total_nbit,
                    total_ncell, *entry)
    b += b"\0" * (PHF_HEADER_BYTES - len(b))
    return b


def phf_segment(codes, bklen=1024, sublen=None, n_cu=256, books=None):
    """The Huffman segment of an archive (hf_buf.cc:111-139,191-211); books = (book, revbook)
    to encode with instead of the reference's codebook of the full histogram."""
    n = codes.size
    if sublen is None:
        sublen, _ = coarse_tune(n, n_cu)
    hist = histogram(codes, bklen)
    book, rv = books if books is not None else codebook(hist, bklen)
    nbit, entry, bs, tot = hf_encode(codes, book, sublen)
    pardeg = nbit.size
    sizes = [PHF_FORCED_ALIGN, rv.size, 4 * pardeg, 4 * pardeg, 4 * bs.size]
    ent = [0]
    for s in sizes:
        ent.append(ent[-1] + s)
    hdr = phf_header_bytes(bklen, sublen, pardeg, n, tot, bs.size, ent)
    seg = hdr + b"\0" * (PHF_FORCED_ALIGN - len(hdr)) + rv.tobytes() + nbit.tobytes() + \
        entry.tobytes() + bs.tobytes()
    assert len(seg) == ent[-1]
    return seg, dict(hist=hist, book=book, revbook=rv, par_nbit=nbit, par_entry=entry,
                     bitstream=bs, sublen=sublen, pardeg=pardeg, total_nbit=tot)


# ------------------------------------------------------------------------ reference
def _ref_outlier_cap(x, y, z):
    """Outlier-list capacity for the reference CPU Lorenzo kernels: they predict every point of a
    partial tile and append outliers with no bound check (lrz.seq.inl:266-284), so the list holds
    the padded tile volume (blocks of 256 / 16 x 16 / 8 x 8 x 8 by dimensionality; a count bound,
    ref_shim.cc padded_points)."""
    up = lambda v, m: (v + m - 1) // m * m  # noqa: E731
    if z > 1:
        return up(x, 8) * up(y, 8) * up(z, 8)
    if y > 1:
        return up(x, 16) * up(y, 16)
    return up(x, 256)


def _ref_count(k):
    if k == 0xFFFFFFFF:
        raise RuntimeError("reference CPU Lorenzo appended more outliers than the list holds")
    return k


def ref_lorenzo_c_f32(data, dims, eb, radius=512):
    data = np.ascontiguousarray(data, np.float32)
    x, y, z = dims
    n = x * y * z
    codes = np.zeros(n, np.uint16)
    cap = _ref_outlier_cap(x, y, z)
    ov = np.zeros(cap, np.float32)
    oi = np.zeros(cap, np.uint32)
    k = _ref_count(ref().ref_c_lorenzo_f32(_ptr(data), x, y, z, eb, radius, _ptr(codes), _ptr(ov), _ptr(oi), cap))
    return codes, ov[:k].copy(), oi[:k].copy()


def ref_lorenzo_c_zz_f32(data, dims, eb, radius=512):
    """Reference CPU ZigZag Lorenzo (CPU_c_lorenzo_nd_with_outlier<f4,true,u2>, lrz.seq.cc:82)."""
    data = np.ascontiguousarray(data, np.float32)
    x, y, z = dims
    n = x * y * z
    codes = np.zeros(n, np.uint16)
    cap = _ref_outlier_cap(x, y, z)
    ov = np.zeros(cap, np.float32)
    oi = np.zeros(cap, np.uint32)
    k = _ref_count(ref().ref_c_lorenzo_zz_f32(_ptr(data), x, y, z, eb, radius, _ptr(codes), _ptr(ov), _ptr(oi), cap))
    return codes, ov[:k].copy(), oi[:k].copy()


def ref_lorenzo3d_f64(data, dims, eb, radius=512):
    """Reference CPU 3-D Lorenzo template (KERNEL_SEQ_c_lorenzo_3d1l, lrz.seq.inl) for double."""
    data = np.ascontiguousarray(data, np.float64)
    x, y, z = dims
    n = x * y * z
    codes = np.zeros(n, np.uint16)
    cap = _ref_outlier_cap(x, y, z)
    ov = np.zeros(cap, np.float32)
    oi = np.zeros(cap, np.uint32)
    k = _ref_count(ref().ref_c_lorenzo3d_f64(_ptr(data), x, y, z, eb, radius, _ptr(codes), _ptr(ov), _ptr(oi), cap))
    return codes, ov[:k].copy(), oi[:k].copy()


def ref_histogram(codes, bklen=1024):
    codes = np.ascontiguousarray(codes, np.uint16)
    h = np.zeros(bklen, np.uint32)
    ref().ref_histogram_u2(_ptr(codes), codes.size, _ptr(h), bklen)
    return h


def ref_codebook(hist, bklen=1024):
    hist = np.ascontiguousarray(hist, np.uint32)
    book = np.zeros(bklen, np.uint32)
    rv = np.zeros(4 * 64 + 2 * bklen, np.uint8)
    nb = ref().ref_build_codebook_u2(_ptr(hist), bklen, _ptr(book), _ptr(rv))
    if nb < 0:
        raise RuntimeError("reference codebook builder threw")
    return book, rv


def ref_time_stages(data, dims, eb, radius=512):
    data = np.ascontiguousarray(data, np.float32)
    ms = np.zeros(4, np.float64)
    ref().ref_time_stages_f32(_ptr(data), dims[0], dims[1], dims[2], eb, radius, _ptr(ms))
    return dict(c_lorenzo=ms[0], histogram=ms[1], codebook=ms[2], x_lorenzo=ms[3])


def ref_time_stages_par(data, slabs, eb, radius=512):
    """slabs: [(offset, (x, y, z))]; one thread per slab, stage clocks started together
    (ref_shim.cc ref_time_stages_par_f32) -> (per-slab stage dicts, wall ms)."""
    data = np.ascontiguousarray(data, np.float32)
    off = np.array([o for o, _ in slabs], np.uint64)
    dims = np.array([d for _, d in slabs], np.uint64).reshape(-1)
    ms = np.zeros(4 * len(slabs), np.float64)
    wall = ref().ref_time_stages_par_f32(_ptr(data), len(slabs), _ptr(off), _ptr(dims), eb, radius, _ptr(ms))
    return [dict(c_lorenzo=ms[4 * i], histogram=ms[4 * i + 1], x_lorenzo=ms[4 * i + 3])
            for i in range(len(slabs))], wall
