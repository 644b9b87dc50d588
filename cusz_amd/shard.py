"""Multi-GPU sharding of the cuSZ hot path (one process per GPU, torch.distributed/RCCL).

The reference has no multi-GPU code.  The path shards naturally because
prediction is tile-local (lrz_c.cuhip.inl: no halo): a slab whose boundaries fall on tile
boundaries -- 8 planes in z (3-D), 32 rows in y (2-D), 1024 elements (1-D) -- yields exactly
the quant codes and outliers the single-GPU run produces for those elements.  Each rank
compresses its slab (or its own independent field) with its own manager: no data-path
collective.  The only exchange is gathering the per-rank archives to a root for output:
sizes by all_gather (8 B per rank), then the archive bytes (padded to the max size) by
all_gather_into_tensor -- over RCCL/xGMI for device tensors, gloo for host tensors.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class Slab:
    rank: int
    offset: int      # first element (linear index into the full field)
    dims: tuple      # (x, y, z) of the slab
    origin: int      # first tile-row index along the split axis (z, y or x in tiles)

    @property
    def count(self) -> int:
        return self.dims[0] * self.dims[1] * self.dims[2]


def tile_extent(dims) -> tuple:
    """(split axis, tile length along it) for the reference tile sizes (launch.hh:47-121)."""
    x, y, z = dims
    if z > 1:
        return 2, 8
    if y > 1:
        return 1, 32
    return 0, 1024


def plan_slabs(dims, world: int):
    """Tile-aligned, as-even-as-possible split of the slowest axis over `world` ranks."""
    dims = tuple(int(v) for v in (tuple(dims) + (1, 1, 1))[:3])
    axis, t = tile_extent(dims)
    length = dims[axis]
    ntiles = (length + t - 1) // t
    out = []
    start_tile = 0
    for r in range(world):
        nt = ntiles // world + (1 if r < ntiles % world else 0)
        lo = min(start_tile * t, length)
        hi = min((start_tile + nt) * t, length)
        d = list(dims)
        d[axis] = hi - lo
        stride = 1
        for a in range(axis):
            stride *= dims[a]
        out.append(Slab(r, lo * stride, tuple(d), start_tile))
        start_tile += nt
    return out


def gather_bytes(buf, dist, root: int = 0):
    """Gather variable-length uint8 tensors (one per rank) to every rank; returns the list on
    `root` (None elsewhere).  Works for cuda tensors over RCCL and cpu tensors over gloo."""
    import torch

    world = dist.get_world_size()
    n = torch.tensor([buf.numel()], dtype=torch.int64, device=buf.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    padded = torch.zeros(mx, dtype=torch.uint8, device=buf.device)
    padded[: buf.numel()] = buf
    out = torch.empty(world * mx, dtype=torch.uint8, device=buf.device)
    dist.all_gather_into_tensor(out, padded) if hasattr(dist, "all_gather_into_tensor") and \
        buf.device.type == "cuda" else dist.all_gather(list(out.view(world, mx).unbind(0)), padded)
    if dist.get_rank() != root:
        return None
    return [out[r * mx: r * mx + sizes[r]] for r in range(world)]


def archive_tensor(ptr: int, nbytes: int, device):
    """Copy a device archive (raw pointer from psz_compress_*) into a torch uint8 tensor."""
    import torch

    from . import hip_memcpy

    t = torch.empty(nbytes, dtype=torch.uint8, device=device)
    hip_memcpy(t.data_ptr(), ptr, nbytes, 3)
    return t
