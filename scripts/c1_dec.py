#!/usr/bin/env python3
"""Config-1 decompress time per Huffman decoder kind (diagnostic): CESM-like 3600x1800 f32,
abs 1e-4; decompress timed by HIP events over 20 calls, output checked against the input."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import cusz_amd as cz  # noqa: E402
from cusz_amd import datagen  # noqa: E402

dims = (3600, 1800, 1)
x = torch.from_numpy(datagen.cesm2d_np(dims[:2], seed=1)).cuda()
s = torch.cuda.current_stream()
r = cz.Resource(cz.F4, dims, stream=s.cuda_stream)
ptr, nb, _ = r.compress(x.data_ptr(), 1e-4)
torch.cuda.synchronize()
y = torch.empty_like(x)
for k in (0, 1, 2):
    r.set_decoder(k)
    r.decompress(ptr, nb, y.data_ptr())
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(20):
        r.decompress(ptr, nb, y.data_ptr())
    e1.record(s)
    torch.cuda.synchronize()
    err = (y.double() - x.double()).abs().max().item()
    print(f"decoder {k}: decompress {e0.elapsed_time(e1) / 20 * 1e3:.1f} us, max err {err:.3e}", flush=True)
