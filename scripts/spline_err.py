#!/usr/bin/env python3
"""Largest |x - x'| / eb of the spline path over the GPU test cases (documents the f32 bound)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import pyoracle  # noqa: E402
import test_gpu_spline as t  # noqa: E402

worst = {}
for dims, dtype, eb in t.CASES:
    data, x, ebx, nol = t._roundtrip(pyoracle, dims, dtype, eb)
    ratio = float(np.max(np.abs(x.astype(np.float64) - data)) / ebx)
    worst[np.dtype(dtype).name] = max(worst.get(np.dtype(dtype).name, 0.0), ratio)
    print(dims, np.dtype(dtype).name, eb, f"max err / eb = {ratio:.6f}")
print("worst", worst)
