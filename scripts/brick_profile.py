#!/usr/bin/env python3
"""Fused brick decoder phase profile (diagnostic): loads the instrumented library
(make -C cusz_amd prof), decompresses a config-2 field and prints per-brick averages of the
phase clocks k_brick3_decode keeps in that build."""
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
eb = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-4
x = datagen.smooth3d_torch(dims, seed=2, device="cuda")
y = torch.empty_like(x)
s = torch.cuda.current_stream()
r = cz.Resource(cz.F4, dims, stream=s.cuda_stream)
ptr, nb, _ = r.compress(x.data_ptr(), eb, cz.Abs)
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
nbk = v[0]
print(f"decompress {ev[0].elapsed_time(ev[1]) / reps * 1e3:.1f} us per call (profiled build), bricks {nbk:.0f}")
names = ["brick", "setup", "decode", "recon"]
for i, nm in zip([1, 2, 3, 4], names):
    print(f"  {nm:7s} {v[i] / nbk:10.0f} cycles/brick")
print(f"  idle    {v[7] / nbk:10.0f} cycles/brick (work counter + tail)")
print(f"  loop iterations {v[5] / nbk:.1f}/brick ({2 * v[5] / nbk / 256:.3f} steps per symbol per lane)")
print(f"  fallback lane-steps {v[6] / nbk:.1f}/brick; ring rows loaded {v[8] / nbk:.1f}/brick")
err = (y.double() - x.double()).abs().max().item()
print(f"max err {err:.3e}")
