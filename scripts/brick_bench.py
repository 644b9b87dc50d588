#!/usr/bin/env python3
"""Micro-benchmark of the fused brick kernels on a config-2 field (512^3 f32, abs 1e-4).

Times compress and decompress with HIP events on the manager's stream (CUSZ_AMD_LIB selects a
variant library, e.g. one built with a timing-experiment switch).
Usage: python scripts/brick_bench.py [--dims 512x512x512] [--reps 10] [--f64] [--codebook stream]
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
    ap.add_argument("--eb", type=float, default=1e-4)
    ap.add_argument("--f64", action="store_true")
    ap.add_argument("--codebook", default="default", choices=["default", "exact", "sampled", "stream"])
    ap.add_argument("--dbg", default="0", help="(ignored; kept for old command lines)")
    a = ap.parse_args()
    dims = tuple(int(v) for v in a.dims.split("x"))
    dt = torch.float64 if a.f64 else torch.float32
    if dims[1] == dims[2] == 1:  # 1-D: the config-3 recipe
        d_in = datagen.hacc1d_torch(dims[0], seed=3).to(dt)
    else:
        d_in = datagen.smooth3d_torch(dims, seed=2, dtype=dt)
    n = d_in.numel()
    out = torch.empty(n, dtype=dt, device="cuda")
    st = torch.cuda.current_stream()
    r = cz.Resource(cz.F8 if a.f64 else cz.F4, dims, stream=st.cuda_stream)
    r.enable_timing(True)
    if a.codebook != "default":
        r.set_codebook({"exact": cz.CODEBOOK_EXACT, "sampled": cz.CODEBOOK_SAMPLED, "stream": cz.CODEBOOK_STREAM}[a.codebook])
    ptr, nb, _ = r.compress(d_in.data_ptr(), a.eb)
    print(f"layout={r.internals().layout} sublen={r.header.vle_sublen} CR={n * d_in.element_size() / nb:.3f}")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timeit(fn):
        fn()
        torch.cuda.synchronize()
        ev[0].record(st)
        for _ in range(a.reps):
            fn()
        ev[1].record(st)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / a.reps

    tc = timeit(lambda: r.compress(d_in.data_ptr(), a.eb))
    stc = r.stage_times()
    ptr, nb, _ = r.compress(d_in.data_ptr(), a.eb)
    torch.cuda.synchronize()
    td = timeit(lambda: r.decompress(ptr, nb, out.data_ptr()))
    print(f"decompress dbg=0: {td * 1e3:.1f} us")
    err = (out.double() - d_in.double()).abs().max().item()
    gb = n * d_in.element_size() / 1e9
    print(f"compress {tc * 1e3:.1f} us ({gb / tc * 1e3:.0f} GB/s); stages ms: predict {stc[cz.T_PREDICT]:.4f} "
          f"book {stc[cz.T_BOOK]:.4f} encode {stc[cz.T_ENCODE]:.4f} finalize {stc[cz.T_FINALIZE]:.4f}")
    print(f"decompress {td * 1e3:.1f} us ({gb / td * 1e3:.0f} GB/s); max err {err:.3e}")


if __name__ == "__main__":
    main()
