"""Multi-GPU sharding of the cuSZ hot path (one process per GPU, torch.distributed/RCCL).

The reference has no multi-GPU code.  The path shards naturally because
prediction is tile-local (lrz_c.cuhip.inl: no halo): a slab whose boundaries fall on tile
boundaries -- 8 planes in z (3-D), 32 rows in y (2-D), 1024 elements (1-D) -- yields exactly
the quant codes and outliers the single-GPU run produces for those elements.

Exchange steps (the only collectives; everything else is rank-local):
  1. optional global codebook: every rank runs pass 1 on its slab
     (psz_amd_compress_scan_*), the u32[bklen] histograms of all fields are summed by ONE
     all-reduce (``allreduce_histograms``: [fields, bklen] int64, 8 KB per field), and every
     rank finishes its slabs with the same codebook (psz_amd_compress_finish);
  2. gather of the per-rank archives to ONE root (``gather_to_root``): 8-B sizes by
     all_gather, then exact-size point-to-point sends to the root (batch_isend_irecv ->
     grouped ncclSend/ncclRecv over xGMI on GPUs, gloo on CPU) -- no max-size padding and no
     bytes to non-root ranks;
  3. the root merges the slabs of one field into the single archive a one-process run would
     have written (``merge``: psz_amd_merge_archives, host code).
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


def gather_to_root(buf, dist, root: int = 0):
    """Gather one variable-length uint8 tensor per rank to `root` only: sizes by all_gather
    (one int64 per rank), bytes by exact-size point-to-point transfers.  Returns the list of
    per-rank tensors (rank order) on `root`, None elsewhere.  Device tensors go over RCCL
    (grouped ncclSend/ncclRecv), host tensors over gloo."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    n = torch.tensor([buf.numel()], dtype=torch.int64, device=buf.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    if rank != root:
        if sizes[rank]:
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, buf.contiguous(), root)]):
                w.wait()
        return None
    out = [buf if r == root else torch.empty(sizes[r], dtype=torch.uint8, device=buf.device)
           for r in range(world)]
    ops = [dist.P2POp(dist.irecv, out[r], r) for r in range(world) if r != root and sizes[r]]
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    return out


def allreduce_histograms(hists, dist):
    """Sum the u32 histograms of every rank's slabs in one all-reduce.  `hists`: [fields, bklen]
    integer tensor (int32 holding the u32 bit pattern on the device for RCCL, int64 on the host
    for gloo); summed in place and returned."""
    dist.all_reduce(hists, op=dist.ReduceOp.SUM)
    return hists


def check_streams(resources, device) -> None:
    """The sharded helpers order their phases by torch's current stream only (no host sync, no
    events): every manager must run on that stream, or the all-reduce could read histograms
    (or extrema) the scans have only partly written.  Raise instead of corrupting silently."""
    import torch

    if device is None or torch.device(device).type != "cuda":
        return
    cur = torch.cuda.current_stream(device).cuda_stream
    for r in resources:
        if getattr(r, "stream", cur) != cur:
            raise ValueError(f"manager stream {r.stream:#x} is not torch's current stream {cur:#x}: "
                             "create the Resource with stream=torch.cuda.current_stream().cuda_stream")


def global_value_ranges(resources, fields, dist):
    """Rel (r2r) mode across slabs: max - min of every field over all ranks.  Each slab's range
    comes from the library's extrema kernel (psz_amd_value_range: extrema.cuhip.inl:150-208, on
    the manager's stream), then ONE all-reduce (MAX) of [fields, 2] = {-min, max}
    (libcusz.cc:287-293 computes this range per field on one GPU)."""
    import torch

    check_streams(resources, fields[0].device)
    mm = torch.empty((len(fields), 2), dtype=torch.float64, device=fields[0].device)
    for i, (r, f) in enumerate(zip(resources, fields)):
        r.value_range(f.data_ptr(), mm[i].data_ptr(), f.numel())
    mm[:, 0].neg_()
    if dist is not None and dist.get_world_size() > 1:
        dist.all_reduce(mm, op=dist.ReduceOp.MAX)
    return [float(hi + lo) for lo, hi in mm.tolist()]


def compress_fields_sharded(resources, fields, eb, dist, mode=0, radius=512, device=None, hists=None):
    """Sharded compress of several fields whose slabs (device tensors `fields`) this rank holds,
    with one codebook per field shared by all ranks: pass 1 per slab, ONE all-reduce of the
    [fields, bklen] histograms, then finish every slab.  Rel mode: eb times the field's global
    value range (one more all-reduce), the slabs then compress with that absolute bound.

    The managers must run on the caller's current stream (torch.cuda.current_stream; checked,
    ValueError otherwise): RCCL orders the all-reduce after the scans and the finish after the
    all-reduce on that stream, so no host synchronisation is needed between the phases.  The u32 histogram sums are
    reduced as int32 (the bit pattern is the u32 sum: every count is < 2^32).
    Each histogram row carries two words after the counts, summed by the same all-reduce: the
    slab's overflow word (outlier cells past its capacity, written by the scan) and a failure
    word.  A rank whose scan fails (e.g. a manager broken by a failed allocation) still joins the
    all-reduce, with a zeroed row and its failure word set, so that no peer waits for it: every
    rank then sees the failure and raises.  A slab with more outliers than its capacity (past the
    reference's 10 %) makes every rank's finish warn through the summed overflow word; every
    rank then repeats its scans, the all-reduce and its finishes once, with the grown capacity.
    A finish that fails otherwise raises after that repeat (which its peers may be waiting for).
    `hists`: optional [fields, 2 radius + 2] int32 scratch on the managers' device (one of
    2 radius + 1 columns is replaced by an internal one).
    Returns [(archive_ptr, nbytes)] (device archives, valid until the manager's next compress)."""
    import torch

    from . import PSZ_AMD_ERR_DEVICE, PSZ_WARN_OUTLIER_TOO_MANY, PszError

    bklen = 2 * radius
    f = len(resources)
    check_streams(resources, device if device is not None else (fields[0].device if fields else None))
    ebs = [eb * r for r in global_value_ranges(resources, fields, dist)] if mode == 1 else [eb] * f
    if hists is None or hists.shape[-1] != bklen + 2:
        hists = torch.empty((f, bklen + 2), dtype=torch.int32, device=device)
    failure = None
    out = []
    for attempt in range(2):
        scan_failed = False
        for i, (r, t) in enumerate(zip(resources, fields)):
            try:
                r.compress_scan(t.data_ptr(), ebs[i], hists[i].data_ptr(), 0, radius)
                hists[i, bklen + 1] = 0
            except PszError as e:
                failure = failure or e
                scan_failed = True
                hists[i].zero_()
                hists[i, bklen + 1] = 1  # this rank's scan failed: the peers learn it from the sum
        if dist is not None and dist.get_world_size() > 1:
            allreduce_histograms(hists, dist)  # the overflow and failure words are summed with the counts
        out, again = [], False
        for i, r in enumerate(resources if not scan_failed else []):
            try:
                ptr, nb, _ = r.compress_finish(hists[i].data_ptr())
            except PszError as e:
                # a slab had more outliers than its capacity (past the reference's 10 %): every
                # rank sees it through the summed overflow word; the capacity has grown
                if e.status == PSZ_WARN_OUTLIER_TOO_MANY and not attempt:
                    again = True
                    continue
                failure = failure or e
                # any other failure: when the summed overflow word makes the other ranks repeat,
                # this rank repeats with them (their all-reduce would wait for it forever); its
                # scan on the repeat fails too (a broken manager) and tells the peers so
                if not attempt and retry_needed(hists[i], bklen):
                    again = True
                continue
            out.append((ptr, nb))
        # a failed scan anywhere: every rank raises (read after the finishes, which have waited
        # for the device anyway: no extra host synchronisation between the phases)
        if scan_failed or int(hists[:, bklen + 1].max().item()) != 0:
            raise failure or PszError(PSZ_AMD_ERR_DEVICE, "compress_scan on a peer rank")
        if not again:
            break
    if failure is not None:
        raise failure
    return out


def retry_needed(hist_row, bklen: int) -> bool:
    """The summed overflow word of a reduced histogram row (u32[2 radius + 2]: counts, overflow
    word, failure word): nonzero when some slab of this field overflowed its outlier list, so
    every rank repeats the scan."""
    return int(hist_row[bklen].item()) != 0


def merge(parts, full_dims, offsets=None) -> bytes:
    """Merge per-slab archives (host bytes, field order) into the whole field's archive."""
    from . import merge_archives

    return merge_archives(parts, full_dims, offsets)


def archive_tensor(ptr: int, nbytes: int, device):
    """Copy a device archive (raw pointer from psz_compress_*) into a torch uint8 tensor."""
    import torch

    from . import hip_memcpy

    t = torch.empty(nbytes, dtype=torch.uint8, device=device)
    hip_memcpy(t.data_ptr(), ptr, nbytes, 3)
    return t
