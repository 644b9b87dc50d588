#!/usr/bin/env python3
"""Huffman decoder micro-benchmark (diagnostic): compress one field, then time
psz_amd_decode_codes for each decoder kind and check the decoded codes against the
encoder's input codes.  usage: dec_bench.py [DIMS] [EB] [SUBLEN] [KINDS]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import cusz_amd as cz  # noqa: E402
from cusz_amd import datagen  # noqa: E402

dims = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "512x512x512").split("x"))
eb = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-4
sublen = int(sys.argv[3]) if len(sys.argv) > 3 else 0
kinds = [int(k) for k in (sys.argv[4] if len(sys.argv) > 4 else "1,2,3").split(",")]
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
x = datagen.smooth3d_torch(dims, seed=2, device=dev)
s = torch.cuda.current_stream(dev)
r = cz.Resource(cz.F4, dims, stream=s.cuda_stream)
r.enable_timing(True)
if sublen:
    r.set_sublen(sublen)
ptr, nb, _ = r.compress(x.data_ptr(), eb, cz.Abs)
torch.cuda.synchronize()
ino = r.internals()
n = int(ino.len)
ref = torch.empty(n, dtype=torch.int16, device=dev)
cz.hip_memcpy(ref.data_ptr(), ino.d_quant_codes, 2 * n, 3)
torch.cuda.synchronize()
print(f"dims={dims} sublen={ino.sublen} pardeg={ino.pardeg} archive={nb} B CR={4 * n / nb:.3f}", flush=True)
codes = torch.empty(n, dtype=torch.int16, device=dev)
for k in kinds:
    r.set_decoder(k)
    ts = []
    ok = True
    for it in range(8):
        cz.hip_memcpy(ino.d_quant_codes, codes.data_ptr(), 2 * n, 3)  # scramble the destination
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r.decode_codes(ptr)
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
        if it == 0:
            got = torch.empty(n, dtype=torch.int16, device=dev)
            cz.hip_memcpy(got.data_ptr(), ino.d_quant_codes, 2 * n, 3)
            torch.cuda.synchronize()
            ok = bool(torch.equal(got, ref))
            if not ok:
                bad = (got != ref).nonzero()
                print(f"  kind {k}: MISMATCH at {bad.numel()} positions, first {bad[:4].flatten().tolist()}")
    ts = sorted(ts[1:])
    print(f"decoder {k}: median {ts[len(ts) // 2] * 1e3:8.1f} us  min {ts[0] * 1e3:8.1f} us  "
          f"{'OK' if ok else 'WRONG'}  ({2 * n / ts[len(ts) // 2] / 1e6:.1f} GB/s of codes)", flush=True)
r.close()
