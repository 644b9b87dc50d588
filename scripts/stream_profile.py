#!/usr/bin/env python3
"""Phase profile of the single-pass encoder k_brick3_stream (diagnostic): loads the instrumented
library (make -C cusz_amd prof), compresses a config-2 field in the stream mode and prints the
per-wave-brick cycle averages of its phases."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CUSZ_AMD_LIB", os.path.join(ROOT, "cusz_amd", "lib_prof", "libcusz_amd.so"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import cusz_amd as cz  # noqa: E402
from cusz_amd import datagen  # noqa: E402

dims = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "512x512x512").split("x"))
x = datagen.smooth3d_torch(dims, seed=2, device="cuda")
s = torch.cuda.current_stream()
r = cz.Resource(cz.F4, dims, stream=s.cuda_stream)
r.set_codebook(cz.CODEBOOK_STREAM)
r.compress(x.data_ptr(), 1e-4, cz.Abs)
torch.cuda.synchronize()
L = cz.lib()
buf = (C.c_ulonglong * 16)()
L.psz_amd_debug_brick_profile(buf, 1)
reps = 5
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record(s)
for _ in range(reps):
    r.compress(x.data_ptr(), 1e-4, cz.Abs)
ev[1].record(s)
torch.cuda.synchronize()
L.psz_amd_debug_brick_profile(buf, 1)
v = [buf[i] / reps for i in range(16)]
nwb = v[0]
print(f"compress {ev[0].elapsed_time(ev[1]) / reps * 1e3:.1f} us per call (profiled build), wave-bricks {nwb:.0f}")
tot = sum(v[1:9])
for i, nm in [(1, "phase 1"), (2, "bar A + ydiff + book"), (3, "phase 2"), (4, "barrier B"), (5, "pack"),
              (6, "look-back"), (7, "barrier C"), (8, "copy-out")]:
    print(f"  {nm:22s} {v[i] / nwb:10.0f} cycles/wave-brick ({100 * v[i] / tot:5.1f} %)")
