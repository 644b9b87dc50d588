"""Sharding logic (CPU): tile-aligned slabs reproduce the single-field codes exactly, and the
archive gather works over a world_size-2 gloo group."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cusz_amd import datagen
from cusz_amd.shard import gather_bytes, plan_slabs


@pytest.mark.parametrize("dims,world", [((64, 48, 40), 2), ((64, 48, 40), 3), ((64, 48, 41), 4),
                                        ((300, 200, 1), 2), ((100_000, 1, 1), 3), ((16, 16, 8), 2)])
def test_slabs_cover_and_align(dims, world):
    slabs = plan_slabs(dims, world)
    n = int(np.prod(dims))
    assert sum(s.count for s in slabs) == n
    off = 0
    for s in slabs:
        assert s.offset == off
        off += s.count


@pytest.mark.parametrize("dims,world", [((40, 24, 40), 2), ((40, 24, 40), 3), ((130, 70, 1), 2),
                                        ((50_000, 1, 1), 3)])
def test_slab_codes_equal_full_field(oracle, dims, world):
    """Tile independence: concatenated per-slab codes/outliers == single-run codes/outliers."""
    data = datagen.smooth3d_np(dims, 3)
    full_codes, fv, fi = oracle.lorenzo_c(data, dims, 1e-4)
    codes, vals, idxs = [], [], []
    for s in plan_slabs(dims, world):
        if s.count == 0:
            continue
        c, v, i = oracle.lorenzo_c(data[s.offset:s.offset + s.count], s.dims, 1e-4)
        codes.append(c), vals.append(v), idxs.append(i.astype(np.int64) + s.offset)
    np.testing.assert_array_equal(np.concatenate(codes), full_codes)
    np.testing.assert_array_equal(np.concatenate(idxs), fi)
    np.testing.assert_array_equal(np.concatenate(vals), fv)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf = torch.arange(100 + 37 * rank, dtype=torch.int32).to(torch.uint8)
    got = gather_bytes(buf, dist, root=0)
    if rank == 0:
        q.put([g.tolist() for g in got])
    dist.barrier()
    dist.destroy_process_group()


def test_gather_bytes_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=120)
    for p in ps:
        p.join(timeout=60)
    assert [len(g) for g in got] == [100, 137]
    assert got[1] == [v & 0xFF for v in range(137)]
