#!/usr/bin/env python3
"""Drive lpc_sim.cc: encode a field's codes with the oracle, emulate the lane decoder, compare."""
import os, subprocess, sys, tempfile
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, ROOT)
import pyoracle as po
from cusz_amd import datagen
exe = os.path.join(tempfile.gettempdir(), "lpc_sim")
subprocess.check_call(["g++", "-O2", "-g", "-DL2CAP=" + os.environ.get("L2CAP", "2048"), "-o", exe, os.path.join(HERE, "lpc_sim.cc")])
dims = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "128x128x64").split("x"))
sublen = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
eb = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-4
x = datagen.smooth3d_np(dims)
codes = po.lorenzo_c(x, dims, eb)[0]
h = po.histogram(codes)
book, rv = po.codebook(h)
nbit, entry, bs, tot = po.hf_encode(codes, book, sublen)
for pre in (0, 4, 8, 12):
    d = tempfile.mkdtemp()
    open(f"{d}/revbook.bin", "wb").write(bytes(rv))
    nbit.tofile(f"{d}/nbit.bin"); entry.tofile(f"{d}/entry.bin")
    open(f"{d}/bitstream.bin", "wb").write(b"\xAB" * pre + bs.tobytes())
    np.array([codes.size, sublen, 1024, pre], np.uint64).tofile(f"{d}/meta.bin")
    subprocess.check_call([exe, d])
    out = np.fromfile(f"{d}/out.bin", np.uint16)
    bad = np.nonzero(out != codes)[0]
    print(f"pre={pre}: mismatches={bad.size}", bad[:10])

# skewed distributions: deep codes (L2 overflow -> slow path) and a two-symbol book
rng = np.random.default_rng(5)
for name, p in [("geom", 0.5 ** np.arange(1, 30)), ("two", np.array([0.7, 0.3]))]:
    p = p / p.sum()
    sym = rng.choice(p.size, size=300000, p=p).astype(np.uint16) + 400
    sym[:1000] = np.arange(1000) % 1024  # every symbol present
    h = po.histogram(sym)
    book, rv = po.codebook(h)
    nbit, entry, bs, tot = po.hf_encode(sym, book, sublen)
    d = tempfile.mkdtemp()
    open(f"{d}/revbook.bin", "wb").write(bytes(rv))
    nbit.tofile(f"{d}/nbit.bin"); entry.tofile(f"{d}/entry.bin")
    open(f"{d}/bitstream.bin", "wb").write(b"\xAB" * 4 + bs.tobytes())
    np.array([sym.size, sublen, 1024, 4], np.uint64).tofile(f"{d}/meta.bin")
    subprocess.check_call([exe, d])
    out = np.fromfile(f"{d}/out.bin", np.uint16)
    print(name, "mismatches", int((out != sym).sum()))

# Fibonacci counts: depth > 27 before the length limit -> L2 overflow -> slow path
cnts = [1, 1]
while len(cnts) < 28:
    cnts.append(cnts[-1] + cnts[-2])
sym = np.concatenate([np.full(c, 100 + i, np.uint16) for i, c in enumerate(cnts)] +
                     [np.array([7, 9], np.uint16)])
sym = sym[rng.permutation(sym.size)]
h = po.histogram(sym)
book, rv = po.codebook(h)
nbit, entry, bs, tot = po.hf_encode(sym, book, sublen)
d = tempfile.mkdtemp()
open(f"{d}/revbook.bin", "wb").write(bytes(rv))
nbit.tofile(f"{d}/nbit.bin"); entry.tofile(f"{d}/entry.bin")
open(f"{d}/bitstream.bin", "wb").write(bs.tobytes())
np.array([sym.size, sublen, 1024, 0], np.uint64).tofile(f"{d}/meta.bin")
subprocess.check_call([exe, d])
out = np.fromfile(f"{d}/out.bin", np.uint16)
print("fib mismatches", int((out != sym).sum()))
