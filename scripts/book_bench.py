#!/usr/bin/env python3
"""Host codebook build time (cusz_amd/csrc/codebook.cc via tests/host/codebook_shim.cc, g++ -O3)
on the config-2 histogram (tests/golden/config2_hist.npy: the oracle's codes of the 512^3 f32
config-2 field at abs 1e-4, all 1024 symbols used).  Usage: python scripts/book_bench.py [codebook source]"""
import ctypes as C
import os
import subprocess
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    import sys
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "cusz_amd", "csrc", "codebook.cc")
    d = tempfile.mkdtemp()
    so = os.path.join(d, "libcb.so")
    subprocess.run(["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-o", so,
                    os.path.join(ROOT, "tests", "host", "codebook_shim.cc"), src], check=True)
    lib = C.CDLL(so)
    lib.shim_build_codebook.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    h = np.load(os.path.join(ROOT, "tests", "golden", "config2_hist.npy")).astype(np.uint32)
    book = np.zeros(1024, np.uint32)
    rv = np.zeros(4 * 64 + 2048, np.uint8)
    for _ in range(200):
        lib.shim_build_codebook(h.ctypes.data, 1024, book.ctypes.data, rv.ctypes.data)
    n = 2000
    t = time.perf_counter()
    for _ in range(n):
        lib.shim_build_codebook(h.ctypes.data, 1024, book.ctypes.data, rv.ctypes.data)
    dt = (time.perf_counter() - t) / n
    print(f"{os.path.basename(src)}: build_codebook (config-2 histogram, {int((h > 0).sum())} symbols): {dt * 1e6:.2f} us per call "
          f"(incl. ctypes call overhead)")


if __name__ == "__main__":
    main()
