#!/usr/bin/env python3
"""Decoder phase profile (diagnostic): loads the instrumented library (make -C cusz_amd prof),
compresses + decompresses one field and prints per-chunk cycle/step averages per wave."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("CUSZ_AMD_LIB", os.path.join(ROOT, "cusz_amd", "lib_prof", "libcusz_amd.so"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import cusz_amd as cz  # noqa: E402
from cusz_amd import datagen  # noqa: E402

dims = tuple(int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "512x512x512").split("x"))
eb = float(sys.argv[2]) if len(sys.argv) > 2 else 1e-4
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
x = datagen.smooth3d_torch(dims, seed=2, device=dev)
y = torch.empty_like(x)
s = torch.cuda.current_stream(dev)
r = cz.Resource(cz.F4, dims, stream=s.cuda_stream)
r.enable_timing(True)
kind = int(sys.argv[3]) if len(sys.argv) > 3 else 0
if kind:
    r.set_decoder(kind)
for _ in range(3):
    ptr, nb, _ = r.compress(x.data_ptr(), eb, cz.Abs)
    r.decompress(ptr, nb, y.data_ptr())
torch.cuda.synchronize()
L = cz.lib()
buf = (C.c_ulonglong * (4096 * 16))()
L.psz_amd_debug_decode_profile(buf, 4096 * 16)
a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 16).astype(np.float64)
a = a[a[:, 13] > 0]
ch = a[:, 13].sum()
names = ["stage", "steps", "flush", "vmwait", "barrier"] if kind != 2 else ["load", "count", "resync", "emit", "store"]
if kind == 2:
    print(f"wave decoder per chunk: max-lane steps count={a[:,8].sum()/ch:.1f} resync={a[:,9].sum()/ch:.1f} "
          f"emit={a[:,10].sum()/ch:.1f} sync-iterations={a[:,11].sum()/ch:.2f} global-path={a[:,12].sum()/ch:.3f}")
tot = a[:, :5].sum()
print(f"(lane decoder: 'chunks' = waves) waves={len(a)} chunks={int(ch)} chunks/wave={ch/len(a):.1f} decode_ms={r.stage_times()[cz.T_DECODE]:.4f}")
for k, nm in enumerate(names):
    print(f"  {nm:6s} cycles/chunk={a[:, k].sum()/ch:9.0f}  share={a[:, k].sum()/tot:.3f}")
print(f"  loop iterations per wave={a[:,8].mean():.1f} (4 steps each), windows={a[:,9].mean():.1f}")
print(f"  per-wave total cycles: min={a[:, :5].sum(1).min():.0f} max={a[:, :5].sum(1).max():.0f}")

e = (C.c_ulonglong * (65536 * 4))()
L.psz_amd_debug_encode_profile(e, 65536 * 4)
e = np.frombuffer(e, dtype=np.uint64).reshape(65536, 4).astype(np.float64)
e = e[e.sum(1) > 0]
if len(e) == 0:
    sys.exit(0)
print(f"encoder: {len(e)} workgroups profiled, encode_ms={r.stage_times()[cz.T_ENCODE]:.4f}")
for k, nm in enumerate(["setup", "pack", "lookback", "write"]):
    print(f"  {nm:8s} cycles/wg: mean={e[:, k].mean():9.0f} p50={np.median(e[:, k]):9.0f} max={e[:, k].max():9.0f}")
