#!/usr/bin/env python3
"""Sampled-codebook compress micro-benchmark (diagnostic): config-2 field, median stage times of
psz_compress in the exact and the sampled mode (library HIP events), archive sizes."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import cusz_amd as cz  # noqa: E402
from cusz_amd import datagen  # noqa: E402

dims = (512, 512, 512)
x = datagen.smooth3d_torch(dims, seed=2)
r = cz.Resource(cz.F4, dims)
for mode, name in ((cz.CODEBOOK_EXACT, "exact"), (cz.CODEBOOK_SAMPLED, "sampled")):
    r.set_codebook(mode)
    for _ in range(3):
        r.compress(x.data_ptr(), 1e-4)
    r.enable_timing(True)
    ts = []
    for _ in range(10):
        _, nb, _ = r.compress(x.data_ptr(), 1e-4)
        torch.cuda.synchronize()
        ts.append(np.array(r.stage_times()))
    r.enable_timing(False)
    t = np.median(np.array(ts), axis=0) * 1e3
    print(f"{name}: compress {t[cz.T_COMPRESS]:.1f} us (predict/sample {t[cz.T_PREDICT]:.1f}, book {t[cz.T_BOOK]:.1f}, "
          f"encode/single {t[cz.T_ENCODE]:.1f}, finalize {t[cz.T_FINALIZE]:.1f}), archive {nb} B, CR {4 * x.numel() / nb:.3f}")
