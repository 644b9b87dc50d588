#!/usr/bin/env python3
"""Regenerate the committed golden fixtures under tests/golden/.

Run in the development container (needs /root/reference and oracle/_ref built):

    make -C oracle ref && python tests/golden/make_golden.py

Fixtures written (data only -- inputs and expected outputs):

* kat_lorenzo.npz   -- the reference's own known-answer arrays, parsed as data from
                       test/src/detail/correctness.inl (t{1,2,3}_{in,eq,comp_out,decomp_out});
                       sizes 256 (1D), 16x16 (2D), 8x8x8 (3D); they fit inside one GPU tile,
                       so they pin the GPU semantics too.
* ref_lrz3d.npz     -- outputs of the compiled reference CPU Lorenzo-3D
                       (psz/src/kernel/lrz.seq.cc:35-55) on integer-valued inputs at eb=0.5
                       (ebx2_r = 1, so the CPU path's missing round() is the identity and its
                       8^3 tiling equals the GPU's: SURVEY.md §8c item 2).
* ref_codebook.npz  -- histograms and the compiled reference's canonical codebook
                       (codec/hf/src/hf_bk.seq.cc:72-145) for each: book u32[1024], revbook.
* ref_hist.npz      -- codes and the reference serial histogram (hist_generic.seq.cc:17-30).
"""
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle  # noqa: E402

REF = os.environ.get("PSZ_REFERENCE", "/root/reference")


def parse_correctness_inl():
    txt = open(os.path.join(REF, "test/src/detail/correctness.inl")).read()
    out = {}
    for m in re.finditer(r"static const (float|uint16_t) (t\d_\w+)\[\] = \{(.*?)\};", txt, re.S):
        ty, name, body = m.groups()
        body = re.sub(r"//[^\n]*", "", body)
        vals = [float(v) for v in body.replace("\n", " ").split(",") if v.strip()]
        out[name] = np.array(vals, np.float32 if ty == "float" else np.uint16)
    return out


def skewed_hist(rng, n_sym, total, width):
    h = np.zeros(1024, np.uint32)
    c = rng.normal(512, width, total).round().astype(np.int64)
    c = np.clip(c, 1, 1023)
    np.add.at(h, c, 1)
    h[0] = rng.integers(0, 50)
    return h


def main():
    kat = parse_correctness_inl()
    assert set(kat) >= {"t1_in", "t1_eq", "t1_comp_out", "t1_decomp_out", "t3_decomp_out"}, kat.keys()
    np.savez_compressed(os.path.join(HERE, "kat_lorenzo.npz"), **kat)

    rng = np.random.default_rng(20260313)
    # 3D integer-valued field, dims multiples of 8 (the CPU path carries stale tile
    # buffers across partial tiles, lrz.seq.inl:140-150, so only full tiles coincide).
    dims = (40, 24, 16)
    n = dims[0] * dims[1] * dims[2]
    walk = np.cumsum(rng.integers(-3, 4, n)).astype(np.float32)
    walk[rng.integers(0, n, 40)] += rng.integers(-5000, 5000, 40)
    codes, ov, oi = pyoracle.ref_lorenzo_c_f32(walk, dims, 0.5)
    np.savez_compressed(os.path.join(HERE, "ref_lrz3d.npz"), data=walk, dims=np.array(dims),
                        codes=codes, ol_val=ov, ol_idx=oi)

    hists, books, rvbks = [], [], []
    cases = []
    cases.append(skewed_hist(rng, 1024, 200000, 3.0))
    cases.append(skewed_hist(rng, 1024, 50000, 20.0))
    cases.append(skewed_hist(rng, 1024, 3000, 100.0))
    flat = np.zeros(1024, np.uint32)
    flat[100:900] = 7
    cases.append(flat)
    ties = np.zeros(1024, np.uint32)
    ties[rng.choice(1024, 300, replace=False)] = rng.integers(1, 4, 300)
    cases.append(ties)
    two = np.zeros(1024, np.uint32)
    two[[3, 700]] = [5, 9]
    cases.append(two)
    fib = np.zeros(1024, np.uint32)  # Fibonacci depth 25 (< 27): exact reference behaviour
    a, b = 1, 1
    for i in range(26):
        fib[400 + i] = a
        a, b = b, a + b
    cases.append(fib)
    for k in range(5):
        h = np.zeros(1024, np.uint32)
        m = rng.integers(2, 1024)
        idx = rng.choice(1024, m, replace=False)
        h[idx] = rng.integers(1, 1000, m)
        cases.append(h)
    for h in cases:
        book, rv = pyoracle.ref_codebook(h)
        hists.append(h)
        books.append(book)
        rvbks.append(rv)
    np.savez_compressed(os.path.join(HERE, "ref_codebook.npz"), hist=np.stack(hists),
                        book=np.stack(books), revbook=np.stack(rvbks))

    codes = rng.integers(0, 1024, 100000).astype(np.uint16)
    np.savez_compressed(os.path.join(HERE, "ref_hist.npz"), codes=codes,
                        hist=pyoracle.ref_histogram(codes))
    # (round 2; own generator so the fixtures above stay as they were)
    rng2 = np.random.default_rng(20261016)
    # ZigZag (the reference's own f4 instantiation, lrz.seq.cc:82) and f64 (the 3-D template
    # instantiated for double by oracle/ref_shim.cc) on the same kind of integer field
    codes, ov, oi = pyoracle.ref_lorenzo_c_zz_f32(walk, dims, 0.5)
    np.savez_compressed(os.path.join(HERE, "ref_lrz3d_zz.npz"), data=walk, dims=np.array(dims),
                        codes=codes, ol_val=ov, ol_idx=oi)
    walk64 = np.cumsum(rng2.integers(-3, 4, n)).astype(np.float64)
    walk64[rng2.integers(0, n, 40)] += rng2.integers(-5000, 5000, 40)
    codes, ov, oi = pyoracle.ref_lorenzo3d_f64(walk64, dims, 0.5)
    np.savez_compressed(os.path.join(HERE, "ref_lrz3d_f64.npz"), data=walk64, dims=np.array(dims),
                        codes=codes, ol_val=ov, ol_idx=oi)
    print("fixtures written to", HERE)


if __name__ == "__main__":
    main()
