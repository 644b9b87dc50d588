"""cusz_amd -- MI355X-native (gfx950) error-bounded lossy compressor with cuSZ's C API.

The product is the C-ABI shared library ``cusz_amd/lib/libcusz_amd.so`` (HIP kernels +
C++ pipeline, see include/cusz_rev1.h).  This package is a thin ctypes mirror of that
API for tests, bench.py and Python callers; device memory is passed as raw pointers
(e.g. ``torch.Tensor.data_ptr()``).  Importing never falls back to anything: if the
library is missing, :func:`lib` raises.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("CUSZ_AMD_LIB") or os.path.join(HERE, "lib", "libcusz_amd.so")
CLI_PATH = os.path.join(HERE, "bin", "cusz")

# ---- enums (include/c_type.h, include/cusz/type.h) --------------------------------------
F4, F8 = 0, 1
Abs, Rel = 0, 1
Lorenzo, LorenzoZigZag, LorenzoProto, Spline = 0, 1, 2, 3
Huffman, NullCodec = 0, 5
HistogramGeneric, HistogramSparse = 0, 1

PSZ_SUCCESS = 0
PSZ_WARN_RADIUS_TOO_LARGE = 1
PSZ_WARN_OUTLIER_TOO_MANY = 2
PSZ_ABORT_UNSUPPORTED_TYPE = 3
PSZ_ABORT_UNSUPPORTED_DIMENSION = 4
STATUS_NAMES = [
    "PSZ_SUCCESS", "PSZ_WARN_RADIUS_TOO_LARGE", "PSZ_WARN_OUTLIER_TOO_MANY",
    "PSZ_ABORT_UNSUPPORTED_TYPE", "PSZ_ABORT_UNSUPPORTED_DIMENSION", "PSZ_ABORT_NOT_IMPLEMENTED",
    "PSZ_ABORT_NO_SUCH_PREDICTOR", "PSZ_ABORT_NO_SUCH_CODEC", "PSZ_ABORT_TOO_MANY_UNPREDICTABLE",
    "PSZ_ABORT_TOO_MANY_ENC_BREAK",
]

# extensions beyond psz_error_status (include/cusz_amd.h)
PSZ_AMD_ERR_INVALID_ARG, PSZ_AMD_ERR_BAD_ARCHIVE, PSZ_AMD_ERR_DEVICE, PSZ_AMD_ERR_STATE, PSZ_AMD_ERR_ENCODER = (
    100, 101, 102, 103, 104)
EXT_STATUS_NAMES = {100: "PSZ_AMD_ERR_INVALID_ARG", 101: "PSZ_AMD_ERR_BAD_ARCHIVE", 102: "PSZ_AMD_ERR_DEVICE",
                    103: "PSZ_AMD_ERR_STATE", 104: "PSZ_AMD_ERR_ENCODER"}

T_EXTREMA, T_PREDICT, T_BOOK, T_ENCODE, T_FINALIZE, T_COMPRESS = range(6)
T_SCATTER, T_DECODE, T_RECON, T_DECOMPRESS, T_COUNT = 6, 7, 8, 9, 10


class psz_len(C.Structure):
    _fields_ = [("x", C.c_size_t), ("y", C.c_size_t), ("z", C.c_size_t)]


class psz_pipeline(C.Structure):
    _fields_ = [("predictor", C.c_int), ("hist", C.c_int), ("codec1", C.c_int), ("codec2", C.c_int)]


class psz_rc2(C.Structure):
    _fields_ = [("mode", C.c_int), ("eb", C.c_double), ("radius", C.c_uint16)]


class psz_interp_params(C.Structure):
    _fields_ = [("alpha", C.c_double), ("beta", C.c_double), ("use_md", C.c_bool * 6),
                ("use_natural", C.c_bool * 6), ("reverse", C.c_bool * 6), ("auto_tuning", C.c_uint8)]


class psz_header(C.Structure):
    """176-byte archive header, byte layout of psz/include/cusz/header.h:19-48."""
    _fields_ = [("dtype", C.c_int), ("pipeline", psz_pipeline), ("rc", psz_rc2),
                ("vle_sublen", C.c_int), ("vle_pardeg", C.c_int), ("entry", C.c_uint32 * 6),
                ("len", psz_len), ("splen", C.c_size_t), ("user_input_eb", C.c_double),
                ("min_val", C.c_double), ("max_val", C.c_double), ("intp_param", psz_interp_params)]


class psz_amd_internals(C.Structure):
    _fields_ = [("d_quant_codes", C.c_void_p), ("d_hist", C.c_void_p), ("d_book", C.c_void_p),
                ("len", C.c_size_t), ("bklen", C.c_int), ("sublen", C.c_int), ("pardeg", C.c_int),
                ("ndim", C.c_int), ("splen", C.c_size_t), ("archive_capacity", C.c_size_t),
                ("layout", C.c_int), ("brick_width", C.c_int)]


assert C.sizeof(psz_header) == 176, C.sizeof(psz_header)

# every symbol declared in include/*.h that the library defines
EXPORTS = [
    # cusz_rev1.h
    "psz_create_resource_manager", "psz_create_resource_manager_from_CLI",
    "psz_create_resource_manager_from_header", "psz_modify_resource_manager_from_header",
    "psz_release_resource", "psz_compress_float", "psz_compress_double",
    "psz_compress_analyize_float", "psz_decompress_float", "psz_decompress_double",
    # cusz.h
    "psz_create", "psz_create_default", "psz_create_from_context", "psz_create_from_header",
    "psz_release", "psz_compress", "psz_decompress", "psz_clear_buffer", "psz_version",
    "psz_versioninfo", "psz_make_timerecord", "psz_review_comp_time_breakdown",
    "psz_review_comp_time_from_header", "psz_review_decomp_time_from_header",
    "psz_review_compression", "psz_review_decompression",
    # cusz/context.h
    "pszctx_default_values", "pszctx_set_default_values", "pszctx_minimal_workset",
    "pszctx_set_rawlen", "pszctx_set_len", "pszctx_get_len3", "pszctx_create_from_argv",
    "CLI_x", "CLI_y", "CLI_z", "CLI_w", "CLI_radius", "CLI_bklen", "CLI_dtype", "CLI_predictor",
    "CLI_hist", "CLI_codec1", "CLI_codec2", "CLI_mode", "CLI_eb", "CLI_interp_params",
    # cusz/header.h
    "pszheader_len", "pszheader_len_linear", "pszheader_segments", "pszheader_filesize",
    "pszheader_uncompressed_len", "pszheader_compressed_bytes",
    # hf.h
    "phf_encoded_bytes", "phf_coarse_tune_sublen", "phf_coarse_tune", "phf_reverse_book_bytes",
    "phf_version", "phf_versioninfo",
    # cusz_amd.h
    "psz_amd_get_internals", "psz_amd_enable_timing", "psz_amd_stage_times", "psz_amd_set_sublen",
    "psz_amd_decode_codes", "psz_amd_set_decoder", "psz_amd_set_layout", "psz_amd_set_codebook",
    "psz_amd_version", "psz_amd_last_create_status", "psz_amd_build_book_device",
    "psz_amd_compress_scan_float", "psz_amd_compress_scan_double", "psz_amd_compress_finish",
    "psz_amd_merge_archives", "psz_amd_value_range",
]


def build(jobs: int = 8) -> None:
    """Compile the HIP library and CLI in-tree for gfx950 (hipcc; no GPU needed)."""
    subprocess.run(["make", "-s", "-C", HERE, f"-j{jobs}"], check=True)


_lib = None


def lib():
    """Load libcusz_amd.so; raises if it has not been built (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `make -C cusz_amd` (or __graft_entry__.build())")
    # torch (the usual owner of the device buffers) first: its HIP runtime then serves the library
    # too.  Loaded the other way round, the system runtime comes first and torch's device init
    # later fails in that process ("No HIP GPUs are available").
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    P = C.c_void_p
    L.psz_create_resource_manager.restype = P
    L.psz_create_resource_manager.argtypes = [C.c_int, psz_len, psz_pipeline, P]
    L.psz_create_resource_manager_from_header.restype = P
    L.psz_create_resource_manager_from_header.argtypes = [C.POINTER(psz_header), P]
    L.psz_modify_resource_manager_from_header.argtypes = [P, C.POINTER(psz_header)]
    L.psz_release_resource.argtypes = [P]
    for fn in (L.psz_compress_float, L.psz_compress_double):
        fn.restype = C.c_int
        fn.argtypes = [P, psz_rc2, P, C.POINTER(psz_header), C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    L.psz_compress_analyize_float.restype = C.c_int
    L.psz_compress_analyize_float.argtypes = [P, psz_rc2, P, P]
    for fn in (L.psz_decompress_float, L.psz_decompress_double):
        fn.restype = C.c_int
        fn.argtypes = [P, P, C.c_size_t, P]
    L.psz_amd_get_internals.argtypes = [P, C.POINTER(psz_amd_internals)]
    L.psz_amd_enable_timing.argtypes = [P, C.c_int]
    L.psz_amd_stage_times.argtypes = [P, C.POINTER(C.c_float), C.c_int]
    L.psz_amd_set_sublen.argtypes = [P, C.c_int]
    L.psz_amd_decode_codes.argtypes = [P, P]
    L.psz_amd_set_decoder.argtypes = [P, C.c_int]
    L.psz_amd_set_layout.argtypes = [P, C.c_int]
    L.psz_amd_set_codebook.argtypes = [P, C.c_int]
    L.psz_amd_version.restype = C.c_char_p
    for fn in (L.psz_amd_compress_scan_float, L.psz_amd_compress_scan_double):
        fn.restype = C.c_int
        fn.argtypes = [P, psz_rc2, P, P]
    L.psz_amd_compress_finish.restype = C.c_int
    L.psz_amd_compress_finish.argtypes = [P, P, C.POINTER(psz_header), C.POINTER(C.c_void_p),
                                          C.POINTER(C.c_size_t)]
    L.psz_amd_value_range.restype = C.c_int
    L.psz_amd_value_range.argtypes = [P, P, C.c_size_t, P]
    L.psz_amd_merge_archives.restype = C.c_int
    L.psz_amd_merge_archives.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_int,
                                         C.POINTER(C.c_size_t), psz_len, P, C.c_size_t,
                                         C.POINTER(C.c_size_t)]
    L.psz_amd_build_book_device.restype = C.c_int
    L.psz_amd_build_book_device.argtypes = [P, C.c_int, C.c_uint32, P, P, P]
    L.psz_amd_last_create_status.restype = C.c_int
    L.phf_coarse_tune.argtypes = [C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.pszheader_filesize.restype = C.c_size_t
    L.pszheader_filesize.argtypes = [C.POINTER(psz_header)]
    _lib = L
    return L


# Huffman decoder selection (include/cusz_amd.h PSZ_AMD_DECODER_*)
DECODER_AUTO, DECODER_LANE, DECODER_WAVE = 0, 1, 2
# archive layout (PSZ_AMD_LAYOUT_*)
LAYOUT_BRICK, LAYOUT_REFERENCE, LAYOUT_BRICK_FORCE = 0, 1, 2
CODEBOOK_EXACT, CODEBOOK_SAMPLED, CODEBOOK_STREAM = 0, 1, 2  # PSZ_AMD_CODEBOOK_*


class PszError(RuntimeError):
    def __init__(self, status: int, what: str):
        name = STATUS_NAMES[status] if 0 <= status < len(STATUS_NAMES) else EXT_STATUS_NAMES.get(status, str(status))
        super().__init__(f"{what} failed: {name}")
        self.status = status


class Resource:
    """Python mirror of psz_resource (cusz_rev1.h).  Pointers are device addresses."""

    def __init__(self, dtype: int, dims, predictor: int = Lorenzo, stream: int = 0, header: psz_header = None):
        L = lib()
        if header is not None:
            self._h = L.psz_create_resource_manager_from_header(C.byref(header), C.c_void_p(stream))
        else:
            x, y, z = (tuple(dims) + (1, 1, 1))[:3]
            self._h = L.psz_create_resource_manager(
                dtype, psz_len(x, y, z), psz_pipeline(predictor, HistogramGeneric, Huffman, NullCodec),
                C.c_void_p(stream))
        if not self._h:
            raise PszError(L.psz_amd_last_create_status() or PSZ_AMD_ERR_DEVICE, "psz_create_resource_manager")
        self.dtype = dtype if header is None else header.dtype
        self.codebook = CODEBOOK_SAMPLED  # the library's default (psz_amd_set_codebook)
        self.stream = int(stream or 0)  # the manager's HIP stream handle (0: the null stream)
        self.header = psz_header()

    def close(self):
        if self._h:
            lib().psz_release_resource(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def compress(self, d_in: int, eb: float, mode: int = Abs, radius: int = 512):
        L = lib()
        out = C.c_void_p()
        nbytes = C.c_size_t()
        f = L.psz_compress_float if self.dtype == F4 else L.psz_compress_double
        st = f(self._h, psz_rc2(mode, eb, radius), C.c_void_p(d_in), C.byref(self.header), C.byref(out),
               C.byref(nbytes))
        if st not in (PSZ_SUCCESS, PSZ_WARN_RADIUS_TOO_LARGE):
            raise PszError(st, "psz_compress")
        return out.value, nbytes.value, st

    def compress_scan(self, d_in: int, eb: float, d_hist: int, mode: int = Abs, radius: int = 512):
        """Pass 1 of a sharded compress: the slab's histogram u32[2 radius] goes to d_hist, then
        one more word (outlier cells beyond this slab's capacity); d_hist holds 2 radius + 1."""
        f = lib().psz_amd_compress_scan_float if self.dtype == F4 else lib().psz_amd_compress_scan_double
        st = f(self._h, psz_rc2(mode, eb, radius), C.c_void_p(d_in), C.c_void_p(d_hist))
        if st not in (PSZ_SUCCESS, PSZ_WARN_RADIUS_TOO_LARGE):
            raise PszError(st, "psz_amd_compress_scan")
        return st

    def compress_finish(self, d_hist: int = 0):
        """Codebook from the device histogram d_hist (u32[2 radius + 1]: the summed slab histograms
        and overflow words; 0: the slab's own) -> archive.  PszError(PSZ_WARN_OUTLIER_TOO_MANY)
        when a slab overflowed its outlier capacity: repeat scan and finish (it has grown)."""
        out = C.c_void_p()
        nbytes = C.c_size_t()
        st = lib().psz_amd_compress_finish(self._h, C.c_void_p(d_hist or None), C.byref(self.header),
                                           C.byref(out), C.byref(nbytes))
        if st != PSZ_SUCCESS:
            raise PszError(st, "psz_amd_compress_finish")
        return out.value, nbytes.value, st

    def value_range(self, d_in: int, d_minmax: int, n: int = 0):
        """{min, max} of a device field (doubles) -> d_minmax, on the manager's stream (no sync)."""
        st = lib().psz_amd_value_range(self._h, C.c_void_p(d_in), n, C.c_void_p(d_minmax))
        if st != PSZ_SUCCESS:
            raise PszError(st, "psz_amd_value_range")

    def decompress(self, d_archive: int, nbytes: int, d_out: int):
        L = lib()
        f = L.psz_decompress_float if self.dtype == F4 else L.psz_decompress_double
        st = f(self._h, C.c_void_p(d_archive), nbytes, C.c_void_p(d_out))
        if st != PSZ_SUCCESS:
            raise PszError(st, "psz_decompress")

    def set_header(self, h: psz_header):
        lib().psz_modify_resource_manager_from_header(self._h, C.byref(h))

    def internals(self) -> psz_amd_internals:
        o = psz_amd_internals()
        lib().psz_amd_get_internals(self._h, C.byref(o))
        return o

    def enable_timing(self, on: bool = True):
        lib().psz_amd_enable_timing(self._h, int(on))

    def stage_times(self):
        a = (C.c_float * T_COUNT)()
        lib().psz_amd_stage_times(self._h, a, T_COUNT)
        return list(a)

    def set_sublen(self, s: int):
        lib().psz_amd_set_sublen(self._h, s)

    def set_decoder(self, kind: int):
        """0 auto, 1 one lane per chunk, 2 one wave per chunk (PSZ_AMD_DECODER_*)."""
        st = lib().psz_amd_set_decoder(self._h, int(kind))
        if st != PSZ_SUCCESS:
            raise PszError(st, "psz_amd_set_decoder")

    def set_layout(self, layout: int):
        """LAYOUT_BRICK (fused, default when eligible), LAYOUT_REFERENCE (byte-identical) or
        LAYOUT_BRICK_FORCE (bricks also for 2-D fields too small for them to pay)."""
        st = lib().psz_amd_set_layout(self._h, int(layout))
        if st != PSZ_SUCCESS:
            raise PszError(st, "psz_amd_set_layout")

    def set_codebook(self, mode: int):
        """CODEBOOK_EXACT (the reference's heap book on the host: byte-identical archives),
        CODEBOOK_SAMPLED (default: 3-D and 1-D bricks book pass 1's brick sample on the host with
        the two-queue algorithm; spline / sharded finishes build the book on the device) or
        CODEBOOK_STREAM (sampled device book + one predict/pack pass; 3-D brick fields)."""
        st = lib().psz_amd_set_codebook(self._h, int(mode))
        if st != PSZ_SUCCESS:
            raise PszError(st, "psz_amd_set_codebook")
        self.codebook = int(mode)

    def decode_codes(self, d_archive: int):
        st = lib().psz_amd_decode_codes(self._h, C.c_void_p(d_archive))
        if st != PSZ_SUCCESS:
            raise PszError(st, "psz_amd_decode_codes")


_hip = None


def build_book_device(d_hist: int, bklen: int, smooth: int, d_book: int, d_revbook: int, stream: int = 0) -> None:
    """The device codebook (psz_amd_build_book_device): device u32[bklen] histogram (+ smooth per
    bin) -> device book u32[bklen] and reverse book (4 * 64 + 2 * bklen bytes), on `stream`."""
    st = lib().psz_amd_build_book_device(C.c_void_p(d_hist), bklen, smooth, C.c_void_p(d_book),
                                         C.c_void_p(d_revbook), C.c_void_p(stream))
    if st != 0:
        raise PszError(st, "psz_amd_build_book_device")


def hip_memcpy(dst: int, src: int, nbytes: int, kind: int) -> None:
    """hipMemcpy (kind: 1 H2D, 2 D2H, 3 D2D) on raw addresses, e.g. an archive pointer."""
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipMemcpy.restype = C.c_int
    st = _hip.hipMemcpy(C.c_void_p(dst), C.c_void_p(src), nbytes, kind)
    if st != 0:
        raise RuntimeError(f"hipMemcpy failed: {st}")


def merge_archives(parts, full_dims, offsets=None) -> bytes:
    """psz_amd_merge_archives over host byte strings (field order) -> the merged archive."""
    L = lib()
    bufs = [C.create_string_buffer(bytes(p), len(p)) for p in parts]
    ptrs = (C.c_void_p * len(parts))(*[C.cast(b, C.c_void_p) for b in bufs])
    sizes = (C.c_size_t * len(parts))(*[len(p) for p in parts])
    offs = (C.c_size_t * len(parts))(*offsets) if offsets is not None else None
    x, y, z = (tuple(full_dims) + (1, 1, 1))[:3]
    need = C.c_size_t()
    st = L.psz_amd_merge_archives(ptrs, sizes, len(parts), offs, psz_len(x, y, z), None, 0, C.byref(need))
    if st != PSZ_SUCCESS:
        raise PszError(st, "psz_amd_merge_archives")
    out = C.create_string_buffer(need.value)
    st = L.psz_amd_merge_archives(ptrs, sizes, len(parts), offs, psz_len(x, y, z), out, need.value,
                                  C.byref(need))
    if st != PSZ_SUCCESS:
        raise PszError(st, "psz_amd_merge_archives")
    return out.raw[: need.value]


def coarse_tune(n: int):
    s, p = C.c_int(), C.c_int()
    lib().phf_coarse_tune(n, C.byref(s), C.byref(p))
    return s.value, p.value
