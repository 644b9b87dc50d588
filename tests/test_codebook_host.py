"""The library's host codebook builders (cusz_amd/csrc/codebook.cc, compiled here with g++ from
the same source the library links) against the oracle's independent builders (psz_oracle.c):
identical book words and revbook bytes, including trees deeper than 27 bits (length limit) --
the reference heap (exact mode) and the two-queue book of hist + smooth (sampled bricks).
CPU-only."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def shim(tmp_path_factory):
    out = tmp_path_factory.mktemp("cb") / "libcbshim.so"
    src = [os.path.join(ROOT, "tests", "host", "codebook_shim.cc"), os.path.join(ROOT, "cusz_amd", "csrc", "codebook.cc")]
    try:
        subprocess.run(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-o", str(out)] + src, check=True,
                       capture_output=True, timeout=120)
    except (OSError, subprocess.CalledProcessError) as e:
        pytest.skip(f"g++ unavailable: {e}")
    lib = C.CDLL(str(out))
    lib.shim_build_codebook.restype = C.c_int
    lib.shim_build_codebook.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    lib.shim_build_codebook_twoqueue.restype = C.c_int
    lib.shim_build_codebook_twoqueue.argtypes = [C.c_void_p, C.c_int, C.c_uint32, C.c_void_p, C.c_void_p]
    return lib


def _hists():
    rng = np.random.default_rng(7)
    for t in range(300):
        bklen = [1024, 256, int(rng.integers(2, 1025))][t % 3]
        i = np.arange(bklen)
        mode = t % 5
        if mode == 0:
            h = np.where(rng.random(bklen) < 0.25, 0, rng.integers(0, 1000, bklen))
        elif mode == 1:  # Laplacian around the centre (Lorenzo-like), deep tails
            h = np.floor(1e9 * np.exp(-np.abs(i - bklen // 2) / (1.0 + t % 7)))
        elif mode == 2:
            h = rng.integers(0, 3, bklen)
        elif mode == 3:  # Fibonacci-like counts: maximal depth, forces the 27-bit limit
            h = np.minimum(1.618 ** (i % 45), 4e9)
        else:
            h = np.where(rng.random(bklen) < 0.02, rng.integers(1, 1 << 24, bklen), 0)
        yield bklen, np.ascontiguousarray(h, np.uint32)


def test_host_codebook_matches_oracle(shim, oracle):
    deep = 0
    for bklen, h in _hists():
        book = np.zeros(bklen, np.uint32)
        rv = np.zeros(4 * 64 + 2 * bklen, np.uint8)
        nb = shim.shim_build_codebook(h.ctypes.data, bklen, book.ctypes.data, rv.ctypes.data)
        obook, orv = oracle.codebook(h, bklen)
        assert nb == orv.size
        np.testing.assert_array_equal(book, obook)
        np.testing.assert_array_equal(rv, orv)
        deep += int((book[book != 0xFFFFFFFF] >> 27).max(initial=0) == 27)
    assert deep > 0  # the length limit was exercised


def test_host_twoqueue_matches_oracle(shim, oracle):
    deep = 0
    for t, (bklen, h) in enumerate(_hists()):
        smooth = t % 2
        book = np.zeros(bklen, np.uint32)
        rv = np.zeros(4 * 64 + 2 * bklen, np.uint8)
        nb = shim.shim_build_codebook_twoqueue(h.ctypes.data, bklen, smooth, book.ctypes.data, rv.ctypes.data)
        obook, orv = oracle.book_twoqueue(h, bklen, smooth=smooth)
        assert nb == orv.size
        np.testing.assert_array_equal(book, obook)
        np.testing.assert_array_equal(rv, orv)
        deep += int((book[book != 0xFFFFFFFF] >> 27).max(initial=0) == 27)
    assert deep > 0
