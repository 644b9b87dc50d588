#!/usr/bin/env python3
"""Phase clocks of k_chunk_decode (diagnostic): loads the instrumented library (make -C cusz_amd
prof), decompresses a reference-layout field (default: config 1, 3600x1800) and prints per-wave
cycle averages: table build, the whole wave, decode blocks."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CUSZ_AMD_LIB", os.path.join(ROOT, "cusz_amd", "lib_prof", "libcusz_amd.so"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import cusz_amd as cz  # noqa: E402
from cusz_amd import datagen  # noqa: E402

dims = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "3600x1800x1").split("x"))
x = datagen.smooth3d_torch(dims, seed=2, device="cuda")
y = torch.empty_like(x)
s = torch.cuda.current_stream()
r = cz.Resource(cz.F4, dims, stream=s.cuda_stream)
ptr, nb, _ = r.compress(x.data_ptr(), 1e-4, cz.Abs)
r.decompress(ptr, nb, y.data_ptr())
torch.cuda.synchronize()
L = cz.lib()
buf = (C.c_ulonglong * 16)()
L.psz_amd_debug_brick_profile(buf, 1)
reps = 5
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
ev[0].record(s)
for _ in range(reps):
    r.decompress(ptr, nb, y.data_ptr())
ev[1].record(s)
torch.cuda.synchronize()
L.psz_amd_debug_brick_profile(buf, 1)
v = [buf[i] / reps for i in range(16)]
nw = v[13]
print(f"decompress {ev[0].elapsed_time(ev[1]) / reps * 1e3:.1f} us per call (profiled build)")
print(f"waves {nw:.0f}, units {v[0]:.0f}")
print(f"  table build {v[11] / nw:10.0f} cycles/wave")
print(f"  whole wave  {v[12] / nw:10.0f} cycles/wave")
for i, nm in [(1, "start"), (2, "decode"), (3, "drain"), (4, "recon")]:
    print(f"  {nm:7s} {v[i] / max(v[0], 1):10.0f} cycles/unit")
print(f"max err {(y.double() - x.double()).abs().max().item():.3e}")
