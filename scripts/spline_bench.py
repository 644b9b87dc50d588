#!/usr/bin/env python3
"""Micro-benchmark of the spline path on the config-5 field (512^3 f64, r2r 1e-6).

Prints the library's stage times (HIP events on the manager's stream) for compress and
decompress, and the max error.  CUSZ_AMD_LIB selects a variant library (scripts/variants.sh).
Usage: python scripts/spline_bench.py [--dims 512x512x512] [--reps 10] [--f32]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import cusz_amd as cz  # noqa: E402
from cusz_amd import datagen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dims", default="512x512x512")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--eb", type=float, default=1e-6)
    ap.add_argument("--f32", action="store_true")
    a = ap.parse_args()
    dims = tuple(int(v) for v in a.dims.split("x"))
    dt = torch.float32 if a.f32 else torch.float64
    d_in = datagen.smooth3d_torch(dims, seed=5, dtype=dt)
    n = d_in.numel()
    out = torch.empty(n, dtype=dt, device="cuda")
    st = torch.cuda.current_stream()
    r = cz.Resource(cz.F4 if a.f32 else cz.F8, dims, cz.Spline, stream=st.cuda_stream)
    r.enable_timing(True)
    names = {cz.T_EXTREMA: "extrema", cz.T_PREDICT: "spline_c", cz.T_SCATTER: "scatter", cz.T_ENCODE: "encode", cz.T_DECODE: "decode", cz.T_RECON: "spline_x",
             cz.T_COMPRESS: "compress", cz.T_DECOMPRESS: "decompress"}
    acc = {k: 0.0 for k in names}
    for i in range(a.reps + 1):
        ptr, nb, _ = r.compress(d_in.data_ptr(), a.eb, cz.Rel)
        tc = r.stage_times()
        r.decompress(ptr, nb, out.data_ptr())
        td = r.stage_times()
        if i:
            for k in names:
                acc[k] += (tc[k] if k in (cz.T_EXTREMA, cz.T_PREDICT, cz.T_ENCODE, cz.T_COMPRESS) else td[k]) / a.reps
    err = (out.double() - d_in.double()).abs().max().item()
    print(f"CR={n * d_in.element_size() / nb:.3f} err={err:.3e} eb_abs={r.header.rc.eb:.3e} outliers={r.header.splen}")
    print(" ".join(f"{names[k]}={acc[k] * 1e3:.1f}us" for k in names))


if __name__ == "__main__":
    main()
