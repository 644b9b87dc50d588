#!/usr/bin/env python3
"""Decode/encode time and compression ratio against the Huffman chunk length (sublen) on the
config-3 field (1-D HACC-like, 280,953,867 f32) or config 5 (--config 5).  Tuning aid for
pipeline.cc tune_chunking."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import cusz_amd as cz  # noqa: E402
from cusz_amd import datagen  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--sublens", default="0,512,1024,2304")
    a = ap.parse_args()
    if a.config == 3:
        n = 280_953_867
        d = datagen.hacc1d_torch(n, seed=3, device="cuda")
        dims, dt, pred, eb, mode = (n, 1, 1), cz.F4, cz.Lorenzo, 1e-4, cz.Abs
    else:
        dims = (512, 512, 512)
        d = datagen.smooth3d_torch(dims, seed=5, dtype=torch.float64)
        n, dt, pred, eb, mode = d.numel(), cz.F8, cz.Spline, 1e-6, cz.Rel
    out = torch.empty_like(d)
    st = torch.cuda.current_stream()
    for s in [int(v) for v in a.sublens.split(",")]:
        r = cz.Resource(dt, dims, pred, stream=st.cuda_stream)
        r.enable_timing(True)
        if s:
            r.set_sublen(s)
        enc = dec = 0.0
        for i in range(6):
            ptr, nb, _ = r.compress(d.data_ptr(), eb, mode)
            if i:
                enc += r.stage_times()[cz.T_ENCODE] / 5
            r.decompress(ptr, nb, out.data_ptr())
            if i:
                dec += r.stage_times()[cz.T_DECODE] / 5
        err = (out.double() - d.double()).abs().max().item()
        print(f"sublen={r.header.vle_sublen} pardeg={r.header.vle_pardeg} CR={d.element_size() * n / nb:.4f} "
              f"encode={enc * 1e3:.1f}us decode={dec * 1e3:.1f}us err={err:.3e}", flush=True)
        r.close()


if __name__ == "__main__":
    main()
