"""Sharding logic (CPU): tile-aligned slabs reproduce the single-field codes exactly, and the
archive gather works over gloo world sizes 2 and 3."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cusz_amd import datagen
from cusz_amd.shard import plan_slabs
from archive_util import oracle_archive


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


# ---------------------------------------------------------------------------------------------
# Sharded compress with one global codebook: per-rank slab archives merged at
# the root must equal, byte for byte, the archive one process writes for the whole field.
# Per-slab archives are built by the CPU oracle (no GPU here); the exchange (histogram
# all-reduce, gather to root) and the merge are the product code (cusz_amd.shard,
# psz_amd_merge_archives).
def _sharded_worker(rank, world, port, dims, q):
    import sys

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import pyoracle as oracle

    from cusz_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eb = 1e-4
    data = datagen.smooth3d_np(dims, 21)
    s = plan_slabs(dims, world)[rank]
    codes, ov, oi = oracle.lorenzo_c(data[s.offset:s.offset + s.count], s.dims, eb)
    hist = torch.from_numpy(oracle.histogram(codes).astype(np.int64)).reshape(1, -1)
    shard.allreduce_histograms(hist, dist)                      # exchange 1: one all-reduce
    book, rv = oracle.codebook(hist[0].numpy().astype(np.uint32))
    part = oracle_archive(oracle, codes, ov, oi, s.dims, eb, book, rv, sublen=256)
    got = shard.gather_to_root(torch.frombuffer(bytearray(part), dtype=torch.uint8), dist, 0)  # exchange 2
    if rank == 0:
        merged = shard.merge([g.numpy().tobytes() for g in got], dims,
                             [p.offset for p in plan_slabs(dims, world)])
        q.put(merged)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_merged_archive_equals_single_process(oracle, world):
    dims = (64, 40, 48)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + world * 17 + os.getpid() % 500
    ps = [ctx.Process(target=_sharded_worker, args=(r, world, port, dims, q)) for r in range(world)]
    for p in ps:
        p.start()
    merged = q.get(timeout=180)
    for p in ps:
        p.join(timeout=60)
    data = datagen.smooth3d_np(dims, 21)
    codes, ov, oi = oracle.lorenzo_c(data, dims, 1e-4)
    book, rv = oracle.codebook(oracle.histogram(codes))
    single = oracle_archive(oracle, codes, ov, oi, dims, 1e-4, book, rv, sublen=256)
    assert len(merged) == len(single)
    assert merged == single


def _gather_worker(rank, world, port, q):
    from cusz_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    buf = (torch.arange(50 + 91 * rank, dtype=torch.int32) * (rank + 1)).to(torch.uint8)
    got = shard.gather_to_root(buf, dist, root=1)
    q.put((rank, None if got is None else [g.tolist() for g in got]))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_to_root_exact_sizes_gloo_world3():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + os.getpid() % 500
    ps = [ctx.Process(target=_gather_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(3))
    for p in ps:
        p.join(timeout=60)
    assert res[0] is None and res[2] is None  # only the root receives
    assert [len(g) for g in res[1]] == [50, 141, 232]
    assert res[1][2] == [(v * 3) & 0xFF for v in range(232)]


def test_merge_rejects_mismatched_codebooks(oracle):
    import cusz_amd as cz

    dims = (64, 40, 16)
    data = datagen.smooth3d_np(dims, 5)
    parts = []
    for s in plan_slabs(dims, 2):
        codes, ov, oi = oracle.lorenzo_c(data[s.offset:s.offset + s.count], s.dims, 1e-4)
        book, rv = oracle.codebook(oracle.histogram(codes))  # per-slab books: not mergeable
        parts.append(oracle_archive(oracle, codes, ov, oi, s.dims, 1e-4, book, rv, sublen=256))
    with pytest.raises(cz.PszError) as e:
        cz.merge_archives(parts, dims)
    assert e.value.status == cz.PSZ_AMD_ERR_INVALID_ARG


@pytest.mark.parametrize("dims,cut", [((64, 40, 16), 4), ((300, 64, 1), 16), ((4096, 1, 1), 512)])
def test_merge_rejects_slabs_off_tile_boundaries(oracle, dims, cut):
    """A seam that is not on a prediction-tile boundary (z % 8, y % 32, x % 1024) changes the codes
    the whole field would get: the merge must refuse it even with one shared codebook."""
    import cusz_amd as cz

    data = datagen.smooth3d_np(dims, 5)
    axis = 2 if dims[2] > 1 else (1 if dims[1] > 1 else 0)
    stride = int(np.prod(dims[:axis]))
    sizes = [cut, dims[axis] - cut]
    full_codes, _, _ = oracle.lorenzo_c(data, dims, 1e-4)
    book, rv = oracle.codebook(oracle.histogram(full_codes))
    parts, off = [], 0
    for sz in sizes:
        d = list(dims)
        d[axis] = sz
        d = tuple(d)
        cnt = stride * sz
        codes, ov, oi = oracle.lorenzo_c(data[off:off + cnt], d, 1e-4)
        parts.append(oracle_archive(oracle, codes, ov, oi, d, 1e-4, book, rv, sublen=256))
        off += cnt
    with pytest.raises(cz.PszError) as e:
        cz.merge_archives(parts, dims)
    assert e.value.status == cz.PSZ_ABORT_UNSUPPORTED_DIMENSION


def test_merge_rejects_wrong_slab_extent(oracle):
    """Slabs whose faster extents differ from the field's are not slabs of it."""
    import cusz_amd as cz

    dims = (64, 40, 16)
    d = (64, 20, 16)  # two halves along y of a 3-D field: not a z split
    data = datagen.smooth3d_np(d, 5)
    codes, ov, oi = oracle.lorenzo_c(data, d, 1e-4)
    book, rv = oracle.codebook(oracle.histogram(codes))
    p = oracle_archive(oracle, codes, ov, oi, d, 1e-4, book, rv, sublen=256)
    with pytest.raises(cz.PszError) as e:
        cz.merge_archives([p, p], dims)
    assert e.value.status == cz.PSZ_ABORT_UNSUPPORTED_DIMENSION


def test_merge_rejects_truncated_part(oracle):
    """A part shorter than its own header's segment table says is a malformed archive, told apart
    from a well-formed part of the wrong shape by its status."""
    import cusz_amd as cz

    dims = (64, 40, 16)
    data = datagen.smooth3d_np(dims, 5)
    codes, ov, oi = oracle.lorenzo_c(data, dims, 1e-4)
    book, rv = oracle.codebook(oracle.histogram(codes))
    p = oracle_archive(oracle, codes, ov, oi, dims, 1e-4, book, rv, sublen=256)
    for cut in (len(p) - 8, 100):
        with pytest.raises(cz.PszError) as e:
            cz.merge_archives([p[:cut]], dims)
        assert e.value.status == cz.PSZ_AMD_ERR_BAD_ARCHIVE


class _FakeSlab:
    """A manager stand-in for the collective logic of shard.compress_fields_sharded (no GPU):
    the scan writes a histogram row (+ an overflow word), the finish returns a fake archive or
    raises as scripted per attempt."""

    def __init__(self, hists, row, scan_fail=(), finish_status=None, overflow=0):
        self.hists, self.row, self.calls = hists, row, 0
        self.scan_fail, self.finish_status, self.overflow = scan_fail, finish_status or {}, overflow

    def compress_scan(self, ptr, eb, hist_ptr, mode, radius):
        from cusz_amd import PSZ_AMD_ERR_DEVICE, PszError

        k = self.calls
        self.calls += 1
        if k in self.scan_fail:
            raise PszError(PSZ_AMD_ERR_DEVICE, "compress_scan")
        bklen = 2 * radius
        self.hists[self.row, :bklen] = 1
        self.hists[self.row, bklen] = self.overflow if k == 0 else 0

    def compress_finish(self, hist_ptr):
        from cusz_amd import PszError

        st = self.finish_status.get(self.calls - 1)
        if st is not None:
            raise PszError(st, "compress_finish")
        return 1234, 56, None


def _retry_worker(rank, world, port, case, q):
    from cusz_amd import PSZ_AMD_ERR_DEVICE, PSZ_WARN_OUTLIER_TOO_MANY
    from cusz_amd import shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    radius = 4
    hists = torch.zeros((1, 2 * radius + 2), dtype=torch.int32)
    if case == "scan_fails":  # rank 1's manager is broken: its scan fails before the all-reduce
        r = _FakeSlab(hists, 0, scan_fail=(0,) if rank == 1 else ())
    elif case == "overflow":  # rank 0's slab overflows: every rank warns, both repeat, then succeed
        st = {0: PSZ_WARN_OUTLIER_TOO_MANY}
        r = _FakeSlab(hists, 0, finish_status=st, overflow=5 if rank == 0 else 0)
    else:  # "finish_fails": rank 0's finish fails hard while the overflow makes rank 1 repeat;
        # rank 0 repeats too, its scan then fails (a broken manager), and both raise
        st = {0: PSZ_AMD_ERR_DEVICE if rank == 0 else PSZ_WARN_OUTLIER_TOO_MANY}
        r = _FakeSlab(hists, 0, scan_fail=(1,) if rank == 0 else (), finish_status=st, overflow=3 if rank == 1 else 0)
    x = torch.zeros(8)
    try:
        out = shard.compress_fields_sharded([r], [x], 1e-4, dist, radius=radius, hists=hists)
        q.put((rank, "ok", len(out), r.calls))
    except Exception as e:  # noqa: BLE001
        q.put((rank, "raised", getattr(e, "status", None), r.calls))
    dist.destroy_process_group()


@pytest.mark.parametrize("case", ["scan_fails", "overflow", "finish_fails"])
def test_sharded_retry_is_collective(case):
    """No rank waits forever in the histogram all-reduce: a rank whose scan fails still joins it
    and every rank raises; an overflow repeats on every rank together."""
    from cusz_amd import PSZ_AMD_ERR_DEVICE

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29800 + {"scan_fails": 0, "overflow": 7, "finish_fails": 13}[case] + os.getpid() % 500
    ps = [ctx.Process(target=_retry_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(2):
        rank, what, st, calls = q.get(timeout=120)
        res[rank] = (what, st, calls)
    for p in ps:
        p.join(timeout=60)
    if case == "overflow":
        assert res[0] == ("ok", 1, 2) and res[1] == ("ok", 1, 2)
    elif case == "scan_fails":
        assert res[0][0] == "raised" and res[1][0] == "raised"
        assert res[0][1] == PSZ_AMD_ERR_DEVICE and res[1][1] == PSZ_AMD_ERR_DEVICE
    else:
        assert res[0][:2] == ("raised", PSZ_AMD_ERR_DEVICE) and res[1][:2] == ("raised", PSZ_AMD_ERR_DEVICE)
        assert res[0][2] == 2 and res[1][2] == 2  # both repeated the scan once
