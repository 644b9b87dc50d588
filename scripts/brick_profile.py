#!/usr/bin/env python3
"""Phase profile of the fused brick decoder (diagnostic): loads the instrumented library
(make -C cusz_amd prof), decompresses a config-2 field and prints per-brick cycle averages."""
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
x = (datagen.hacc1d_torch(dims[0], seed=3) if dims[1] == dims[2] == 1 else
     datagen.smooth3d_torch(dims, seed=2, device="cuda"))
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
nbk = v[0]
print(f"decompress {ev[0].elapsed_time(ev[1]) / reps * 1e3:.1f} us per call (profiled build), bricks (1-D: unit phases) {nbk:.0f}")
for i, nm in [(1, "start"), (2, "decode"), (3, "drain"), (4, "recon")]:
    print(f"  {nm:7s} {v[i] / nbk:10.0f} cycles/brick")
print(f"  loop iterations {v[5] / nbk:.1f}/brick ({v[5] / nbk * 2 * 4:.0f} wave-steps, kF = 4)")
print(f"  3-D: quarters {v[6] / nbk:.1f}/brick, with a long code {v[7] / nbk:.1f}/brick; 1-D lane-steps: done {v[7] / nbk:.0f}/brick, starved {v[6] / nbk:.0f}/brick")
if v[10]:
    print(f"  3-D ring refill waits {v[10] / nbk:.0f} cycles/brick")
if v[9] and not v[10]:
    print(f"  3-D lane-quarters: wanting {v[9] / nbk:.0f}/brick, starved {v[8] / nbk:.0f}/brick")
elif v[8] or v[9]:
    print(f"  1-D recon: values {v[8] / nbk:.0f}, scans + stores {v[9] / nbk:.0f} cycles/brick")
print(f"max err {(y.double() - x.double()).abs().max().item():.3e}")
