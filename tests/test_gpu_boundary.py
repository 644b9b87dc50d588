"""Behavioural tests of the drop-in boundary: the `cusz` CLI round trip
(cli.cc:51-172: -z writes FILE.cusza, -x writes FILE.cuszx, --origin reports the max error)
and the older cusz.h compressor API (libcusz.cc:119-214), both against the resource-manager
API's archive for the same input."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest
import torch

import cusz_amd as cz
from cusz_amd import datagen
from gpu_util import d2h, sync, to_device

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("dims,dtype,mode,pred", [((256, 48, 40), "f32", "abs", "lrz"),
                                                  ((96, 64, 24), "f32", "abs", "lrz"),
                                                  ((3000, 100, 1), "f32", "abs", "lrz"),
                                                  ((256, 32, 16), "f64", "r2r", "lrz-zz")])
def test_cli_roundtrip(tmp_path, dims, dtype, mode, pred):
    npdt = np.float32 if dtype == "f32" else np.float64
    data = datagen.smooth3d_np(dims, 4, dtype=npdt) if dims[2] > 1 else datagen.cesm2d_np(dims[:2], 4, dtype=npdt)
    f = tmp_path / "field.bin"
    data.tofile(f)
    eb = 1e-4
    lens = "x".join(str(d) for d in dims if d > 1) if dims[2] > 1 else f"{dims[0]}x{dims[1]}"
    z = subprocess.run([cz.CLI_PATH, "-z", "-t", dtype, "-m", mode, "-e", str(eb), "-l", lens, "-p", pred,
                        "-i", str(f)], capture_output=True, text=True, timeout=120)
    assert z.returncode == 0, z.stderr
    arch = (tmp_path / "field.bin.cusza").read_bytes()
    # the archive file is the C API's archive for the same input (and carries its header)
    r = cz.Resource(cz.F4 if dtype == "f32" else cz.F8, dims,
                    cz.LorenzoZigZag if pred == "lrz-zz" else cz.Lorenzo)
    d = to_device(data)
    ptr, nb, _ = r.compress(d.data_ptr(), eb, cz.Rel if mode == "r2r" else cz.Abs)
    assert d2h(ptr, nb).tobytes() == arch
    x = subprocess.run([cz.CLI_PATH, "-x", "-i", str(tmp_path / "field.bin.cusza"), "--origin", str(f)],
                       capture_output=True, text=True, timeout=120)
    assert x.returncode == 0, x.stderr
    out = np.fromfile(tmp_path / "field.bin.cuszx", dtype=npdt)
    eb_abs = eb * (float(data.max()) - float(data.min())) if mode == "r2r" else eb
    ulp = (2.0 ** -23 if dtype == "f32" else 2.0 ** -52) * float(np.abs(data).max())
    assert np.abs(out.astype(np.float64) - data).max() <= 1.001 * eb_abs + ulp
    m = re.search(r"max-error ([0-9.e+-]+)", x.stdout)
    assert m and float(m.group(1)) <= 1.001 * eb_abs + ulp, x.stdout


class psz_len3(C.Structure):
    _fields_ = [("x", C.c_size_t), ("y", C.c_size_t), ("z", C.c_size_t)]


def test_legacy_api_roundtrip():
    L = cz.lib()
    L.psz_create_default.restype = C.c_void_p
    L.psz_create_default.argtypes = [C.c_int, psz_len3]
    L.psz_compress.restype = C.c_int
    L.psz_compress.argtypes = [C.c_void_p, C.c_void_p, psz_len3, C.c_double, C.c_int, C.POINTER(C.c_void_p),
                               C.POINTER(C.c_size_t), C.c_void_p, C.c_void_p, C.c_void_p]
    L.psz_decompress.restype = C.c_int
    L.psz_decompress.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, psz_len3, C.c_void_p, C.c_void_p]
    L.psz_release.argtypes = [C.c_void_p]
    dims = (256, 40, 24)
    data = datagen.smooth3d_np(dims, 9)
    d = to_device(data)
    comp = L.psz_create_default(cz.F4, psz_len3(*dims))
    assert comp
    out, nb = C.c_void_p(), C.c_size_t()
    # header == NULL: decompress must still find the compress header
    st = L.psz_compress(comp, d.data_ptr(), psz_len3(*dims), 1e-4, cz.Abs, C.byref(out), C.byref(nb), None, None, None)
    assert st == cz.PSZ_SUCCESS
    ref = cz.Resource(cz.F4, dims)
    p2, n2, _ = ref.compress(d.data_ptr(), 1e-4)
    a_leg, a_api = d2h(out.value, nb.value).tobytes(), d2h(p2, n2).tobytes()
    assert a_leg[176:] == a_api[176:]  # same segments; header fields the legacy context sets may differ
    h_leg, h_api = cz.psz_header.from_buffer_copy(a_leg[:176]), cz.psz_header.from_buffer_copy(a_api[:176])
    assert list(h_leg.entry) == list(h_api.entry) and h_leg.splen == h_api.splen and h_leg.rc.eb == h_api.rc.eb
    o = torch.full((data.size,), float("nan"), device="cuda")
    st = L.psz_decompress(comp, out.value, nb.value, o.data_ptr(), psz_len3(*dims), None, None)
    sync()
    assert st == cz.PSZ_SUCCESS
    assert np.abs(o.cpu().numpy().astype(np.float64) - data).max() <= 1.001e-4
    L.psz_release(comp)


def test_decompress_rejects_truncated_archive():
    dims = (256, 16, 16)
    data = datagen.smooth3d_np(dims, 1)
    r = cz.Resource(cz.F4, dims)
    ptr, nb, _ = r.compress(to_device(data).data_ptr(), 1e-4)
    o = torch.empty(data.size, device="cuda")
    with pytest.raises(cz.PszError):
        r.decompress(ptr, nb - 8, o.data_ptr())  # in_len shorter than the header's entry[5]


@pytest.mark.parametrize("dims", [(512, 24, 16), (300, 200, 1)])
def test_cli_dump_hist_quant(oracle, tmp_path, dims):
    """`--dump quant,hist` (compressor.inl:507-529): <input>.<mode>_<eb>.bk_<2r>.ht_u4 holds the
    histogram and .qt_u2 the quant codes in index order (both layouts), equal to the oracle's."""
    data = datagen.smooth3d_np(dims, 5) if dims[2] > 1 else datagen.cesm2d_np(dims[:2], 5)
    f = tmp_path / "field.bin"
    data.tofile(f)
    lens = "x".join(str(d) for d in dims if d > 1)
    z = subprocess.run([cz.CLI_PATH, "-z", "-t", "f32", "-m", "abs", "-e", "1e-4", "-l", lens, "-i", str(f),
                        "--dump", "quant,hist"], capture_output=True, text=True, timeout=120)
    assert z.returncode == 0, z.stderr
    codes, _, _ = oracle.lorenzo_c(data, dims, 1e-4)
    base = str(f) + ".abs_1e-4.bk_1024"
    hist = np.fromfile(base + ".ht_u4", dtype=np.uint32)
    np.testing.assert_array_equal(hist, oracle.histogram(codes))
    q = np.fromfile(base + ".qt_u2", dtype=np.uint16)
    np.testing.assert_array_equal(q, codes)
