"""Synthetic inputs of the BASELINE configs, deterministic per seed.

There is no network access, so SDRBench fields (CESM, HACC, Nyx) are replaced by fields
of the same shape and regime.  Small fields are generated with numpy on the host; the
512^3 bench field is generated on the device with torch (same formula).
"""
from __future__ import annotations

import numpy as np


def smooth3d_np(dims, seed=2, noise=1e-3, dtype=np.float32):
    """config 2 formula: sin(0.05x)cos(0.07y) + 0.5 sin(0.03z + 0.01x) + noise*N(0,1)."""
    x, y, z = dims
    rng = np.random.default_rng(seed)
    zz, yy, xx = np.meshgrid(np.arange(z), np.arange(y), np.arange(x), indexing="ij")
    f = np.sin(0.05 * xx) * np.cos(0.07 * yy) + 0.5 * np.sin(0.03 * zz + 0.01 * xx)
    f = f + noise * rng.standard_normal(f.shape)
    return f.astype(dtype).ravel()


def cesm2d_np(dims=(3600, 1800), seed=1, dtype=np.float32):
    """config 1: 0.5 + 0.4 sin(0.01x) cos(0.013y) + 1e-3 N(0,1), x fastest."""
    x, y = dims[:2]
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(y), np.arange(x), indexing="ij")
    f = 0.5 + 0.4 * np.sin(0.01 * xx) * np.cos(0.013 * yy) + 1e-3 * rng.standard_normal((y, x))
    return f.astype(dtype).ravel()


def hacc1d_np(n, seed=3, jump=0.05, dtype=np.float32):
    """config 3: wrapped random walk in [0,256) with a `jump` chance of a uniform jump."""
    rng = np.random.default_rng(seed)
    steps = rng.normal(0, 2e-3, n)
    jumps = rng.random(n) < jump
    steps[jumps] = rng.uniform(0, 256, jumps.sum())
    return np.mod(np.cumsum(steps), 256.0).astype(dtype)


def smooth3d_torch(dims, seed=2, noise=1e-3, dtype=None, device="cuda"):
    import torch

    dtype = dtype or torch.float32
    x, y, z = dims
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    xs = torch.arange(x, device=device, dtype=torch.float64)
    ys = torch.arange(y, device=device, dtype=torch.float64)
    out = torch.empty(z * y * x, device=device, dtype=dtype)
    plane = (torch.sin(0.05 * xs)[None, :] * torch.cos(0.07 * ys)[:, None])
    for k in range(z):  # plane by plane keeps the f64 temporaries small
        f = plane + 0.5 * torch.sin(0.03 * k + 0.01 * xs)[None, :]
        f = f + noise * torch.randn((y, x), generator=g, device=device, dtype=torch.float64)
        out[k * x * y:(k + 1) * x * y] = f.reshape(-1).to(dtype)
    return out


def hacc1d_torch(n, seed=3, jump=0.05, device="cuda"):
    """config 3 on the device (same recipe as hacc1d_np, torch's generator)."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(seed)
    steps = torch.randn(n, generator=g, device=device, dtype=torch.float64) * 2e-3
    jumps = torch.rand(n, generator=g, device=device, dtype=torch.float64) < jump
    steps = torch.where(jumps, torch.rand(n, generator=g, device=device, dtype=torch.float64) * 256.0, steps)
    out = torch.remainder(torch.cumsum(steps, 0), 256.0).to(torch.float32)
    del steps, jumps
    return out


def nyx_fields_torch(dims, seeds=range(10, 16), device="cuda", z0=0, z1=None):
    """config 4: six Nyx-like fields -- log-normal density exp(0.5 G), three
    velocities 200 G, temperature 1e4 exp(0.3 G), a sixth log-normal -- where G is a smooth
    field (32 seeded plane waves) + 1e-3 noise.  Planes [z0, z1) only (a rank's slab); the noise
    of plane z comes from its own generator, so a slab equals the same planes of the whole field."""
    import torch

    x, y, z = dims
    z1 = z if z1 is None else z1
    out = []
    xs = torch.arange(x, device=device, dtype=torch.float64)
    ys = torch.arange(y, device=device, dtype=torch.float64)
    for i, s in enumerate(seeds):
        g = torch.Generator(device=device)
        g.manual_seed(s)
        k = torch.rand((32, 3), generator=g, device=device, dtype=torch.float64) * 0.2
        ph = torch.rand(32, generator=g, device=device, dtype=torch.float64) * 6.283
        f = torch.empty((z1 - z0) * y * x, device=device, dtype=torch.float32)
        step = 16
        for c0 in range(z0, z1, step):
            c1 = min(z1, c0 + step)
            zs = torch.arange(c0, c1, device=device, dtype=torch.float64)
            G = torch.zeros((c1 - c0, y, x), device=device, dtype=torch.float64)
            for j in range(32):
                G += torch.sin(k[j, 0] * xs[None, None, :] + k[j, 1] * ys[None, :, None] + k[j, 2] * zs[:, None, None]
                               + ph[j])
            G /= 4.0
            for zi in range(c0, c1):
                gn = torch.Generator(device=device)
                gn.manual_seed(s * 100003 + zi)
                G[zi - c0] += 1e-3 * torch.randn((y, x), generator=gn, device=device, dtype=torch.float64)
            if i == 0:
                v = torch.exp(0.5 * G)
            elif i < 4:
                v = 200.0 * G
            elif i == 4:
                v = 1e4 * torch.exp(0.3 * G)
            else:
                v = torch.exp(0.5 * G) * 0.1
            f[(c0 - z0) * x * y:(c1 - z0) * x * y] = v.reshape(-1).to(torch.float32)
        out.append(f)
    return out
