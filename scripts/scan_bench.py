#!/usr/bin/env python3
"""Pass-1 micro-benchmark (diagnostic): times psz_amd_compress_scan (predict + histograms +
outliers + codes) on the config-2 field with HIP events on the manager's stream."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import cusz_amd as cz  # noqa: E402
from cusz_amd import datagen  # noqa: E402

dims = (512, 512, 512)
x = datagen.smooth3d_torch(dims, seed=2)
st = torch.cuda.current_stream()
r = cz.Resource(cz.F4, dims, stream=st.cuda_stream)
hist = torch.zeros(1025, dtype=torch.int32, device="cuda")  # counts + overflow word
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]


def finish():
    try:  # a timing-experiment variant may write an unusable plan: only pass 1 is timed
        r.compress_finish(hist.data_ptr())
    except cz.PszError:
        pass


for _ in range(3):
    r.compress_scan(x.data_ptr(), 1e-4, hist.data_ptr())
    finish()
torch.cuda.synchronize()
ts = []
for _ in range(10):
    ev[0].record(st)
    r.compress_scan(x.data_ptr(), 1e-4, hist.data_ptr())
    ev[1].record(st)
    torch.cuda.synchronize()
    ts.append(ev[0].elapsed_time(ev[1]) * 1e3)
    finish()
    torch.cuda.synchronize()
ts.sort()
print(f"scan {ts[len(ts) // 2]:.1f} us (min {ts[0]:.1f})")
