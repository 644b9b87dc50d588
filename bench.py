#!/usr/bin/env python3
"""bench.py -- device-resident compress+decompress throughput of cusz_amd on MI355X.

Metric (BASELINE.json): "device-resident compress+decompress GB/s (input bytes),
512^3 f32 abs eb=1e-4".  One step = compress + decompress of ONE 512^3 f32 field already
resident in HBM (config 2 of BASELINE.json: Lorenzo-3D + histogram + Huffman), through the
C-ABI.  value = field bytes / step time (max over ranks).

GPUs (one process per GPU).  `--gpus N` with N > 1 and no WORLD_SIZE in the environment
re-launches this script under torch.distributed.run (before any GPU call in the parent); under
torchrun WORLD_SIZE must equal N.  The path partitions into independent fields / tiles (SURVEY.md
§8e), so by default (`--scaling weak`) every rank compresses and decompresses its OWN 512^3 field
(the config's recipe, seed per rank) with no collective in the timed steps; value = N x field
bytes / the slowest rank's step time.  The per-rank archives are then gathered to rank 0 (exact-
size grouped ncclSend/ncclRecv over xGMI) outside the timed steps (host_phases_ms.gather,
value_incl_gather), and the root decompresses every rank's archive against that rank's field.
`--scaling strong` splits ONE field into tile-aligned z-slabs (8-plane multiples,
shard.plan_slabs) instead, and a step is the sharded compress of SURVEY.md §8e:
  pass 1 per slab (psz_amd_compress_scan_float) -> ONE all-reduce of the u32[1024 + 1] histogram
  (RCCL) -> finish per slab with the shared codebook (psz_amd_compress_finish) -> every rank
  decompresses its own slab (its archive stays resident on its GPU).
The gather of the per-rank archives to rank 0 (exact-size grouped ncclSend/ncclRecv over xGMI) is
output collection, outside the timed steps: timed in the host-phase pass (host_phases_ms.gather,
value_incl_gather) and done once before the root merges the slabs into the whole field's archive
(psz_amd_merge_archives) and checks that it decompresses within the error bound.  N = 1 is the same step
with no collective.  Barrier + synchronize bracket the timed steps; the max time over ranks is
used.

Extra fields on the JSON line:
  roofline      dominant kernel: algorithmic bytes / its HIP-event duration vs 8 TB/s
  cpu_baseline  the reference's own CPU path (compiled from /root/reference into
                oracle/_ref; 1 thread, plus an all-core variant) timed on this host, N = 1 only
  stages_ms     per-stage device times (HIP events in the library), rank 0
  phases_ms     per-step host-clock split: compress (incl. all-reduce), gather, decompress
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
METRICS = {
    1: "device-resident compress+decompress GB/s (input bytes), CESM-like 3600x1800 f32 abs eb=1e-4",
    2: "device-resident compress+decompress GB/s (input bytes), 512³ f32 abs eb=1e-4",
    3: "device-resident compress+decompress GB/s (input bytes), HACC-like 1-D 280,953,867 f32 abs eb=1e-4",
    4: "aggregate sharded compress GB/s (input bytes), Nyx-like 6x512³ f32 abs eb=1e-4, z-slabs per rank",
    5: "device-resident compress+decompress GB/s (input bytes), 512³ f64 spline r2r eb=1e-6",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5],
                    help="BASELINE.json config: 2 (default, the metric's workload) = 512^3 f32 Lorenzo; "
                         "1 = CESM-like 3600x1800 f32; 3 = HACC-like 1-D f32 280,953,867; "
                         "4 = Nyx-like 6x512^3 f32 sharded in z-slabs over the ranks (global codebook, "
                         "gather to root); 5 = 512^3 f64 cuSZ-i spline, r2r 1e-6")
    ap.add_argument("--dims", default=None)
    ap.add_argument("--eb", type=float, default=None)
    ap.add_argument("--rotate", type=int, default=3,
                    help="distinct input fields the timed loop cycles through (different seeds), so that no "
                         "step reads an input the previous steps left in the 256 MiB Infinity Cache; "
                         "the same-field rate is reported beside it")
    ap.add_argument("--rel", action="store_true", help="config 4: value-range relative bound (r2r) instead of abs")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="N > 1: weak = an independent field per rank (the default: the path partitions, no "
                         "collective in the timed steps); strong = one field in z-slabs with a shared codebook")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory (PCIe) path timing")
    ap.add_argument("--profile-only", action="store_true", help="few steps, no baselines (rocprof)")
    ap.add_argument("--no-other-modes", action="store_true", help="skip the other codebook modes' timings")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="N > 1 process group: nccl (= RCCL over xGMI); gloo is a diagnostic to rehearse the "
                         "multi-rank path with several ranks on ONE GPU (collectives staged through host memory)")
    ap.add_argument("--dry-run", action="store_true",
                    help="no GPU: exercise the launch, rank plumbing and the collectives (gloo) only")
    return ap.parse_args()


def spawn(args) -> int:
    """One process per GPU: re-run this script under torch.distributed.run.  Called before
    anything in this process touches the GPU (a child process, never an exec)."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main() -> int:
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    if args.dry_run:
        return dry_run(args, world, rank)
    import torch

    dist = None
    if world > 1:
        import torch.distributed as dist

        torch.cuda.set_device(local % torch.cuda.device_count())  # (gloo rehearsal: ranks may share a GPU)
        dist.init_process_group(args.backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    try:
        if args.config == 4:
            bench_sharded(args, world, rank, dist, dev)
        else:
            bench_field(args, world, rank, dist, dev)
    finally:
        if dist is not None:
            dist.destroy_process_group()
    return 0


def dry_run(args, world, rank) -> int:
    """CPU rehearsal of the multi-rank step: gloo process group, the histogram all-reduce and the
    exact-size gather to the root of the GPU path (cusz_amd.shard), on stand-in tensors."""
    import torch

    from cusz_amd import shard

    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
    slab = shard.plan_slabs((512, 512, 512), world)[rank]
    hist = torch.full((1, 1024), slab.count // 1024, dtype=torch.int64)
    if dist is not None:
        shard.allreduce_histograms(hist, dist)
    part = torch.full((1000 + 7 * rank,), rank, dtype=torch.uint8)
    got = shard.gather_to_root(part, dist, 0) if dist is not None else [part]
    ok = int(hist.sum().item()) == 1024 * sum(s.count // 1024 for s in shard.plan_slabs((512, 512, 512), world))
    if rank == 0:
        ok = ok and [g.numel() for g in got] == [1000 + 7 * r for r in range(world)]
        print(json.dumps({"metric": METRICS[args.config], "value": None, "unit": "GB/s", "n_gpus": world,
                          "steps": 0, "warmup": 0, "dry_run": True, "collectives_ok": bool(ok),
                          "slab_planes": [s.dims[2] for s in shard.plan_slabs((512, 512, 512), world)]}),
              flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return 0 if ok else 1


class _DevBytes:
    """Zero-copy view of a device archive (raw pointer from psz_compress_*) for torch."""

    def __init__(self, ptr: int, nbytes: int):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False),
                                         "version": 2, "strides": None}


def archive_view(ptr, nbytes, dev, scratch):
    """The archive as a uint8 tensor for RCCL: zero-copy when torch accepts the array interface,
    else a device-to-device copy into `scratch` (resized on demand)."""
    import torch

    import cusz_amd as cz

    try:
        t = torch.as_tensor(_DevBytes(ptr, nbytes), device=dev)
        if t.data_ptr() == ptr:
            return t, scratch
    except Exception:
        pass
    if scratch is None or scratch.numel() < nbytes:
        scratch = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    cz.hip_memcpy(scratch.data_ptr(), ptr, nbytes, 3)
    return scratch[:nbytes], scratch


def bench_field(args, world, rank, dist, dev):
    import numpy as np
    import torch

    import cusz_amd as cz
    from cusz_amd import datagen, shard

    cfg = {1: ("3600x1800", 1e-4, cz.Abs, cz.Lorenzo, torch.float32),
           2: ("512x512x512", 1e-4, cz.Abs, cz.Lorenzo, torch.float32),
           3: ("280953867", 1e-4, cz.Abs, cz.Lorenzo, torch.float32),
           5: ("512x512x512", 1e-6, cz.Rel, cz.Spline, torch.float64)}[args.config]
    dims = tuple(int(v) for v in (args.dims or cfg[0]).lower().split("x"))
    dims = (dims + (1, 1))[:3]
    args.eb = args.eb if args.eb is not None else cfg[1]
    mode, predictor, tdt = cfg[2], cfg[3], cfg[4]
    esz = 8 if tdt == torch.float64 else 4
    n_full = dims[0] * dims[1] * dims[2]
    # weak scaling (the default): an independent field per rank.  strong: one field in z-slabs --
    # not for spline (its archive has an anchor segment the slab merge does not rebase)
    sharded = world > 1 and predictor != cz.Spline and args.scaling == "strong"
    weak = world > 1 and not sharded
    slab = shard.plan_slabs(dims, world)[rank] if sharded else shard.Slab(rank, 0, dims, 0)
    my_dims, n = slab.dims, slab.count
    seed = {1: 1, 2: 2, 3: 3, 5: 5}[args.config] + (rank if weak else 0)

    def make_field(sd):
        if args.config == 1:
            return torch.from_numpy(datagen.cesm2d_np(dims[:2], seed=sd)).to(dev)
        if args.config == 3:
            return datagen.hacc1d_torch(n_full, seed=sd, device=dev)
        return datagen.smooth3d_torch(dims, seed=sd, dtype=tdt, device=dev)

    d_full = make_field(seed)
    d_in = d_full[slab.offset:slab.offset + n].clone() if sharded else d_full
    if sharded and rank != 0:
        del d_full  # the root keeps the whole field to validate the merged archive
    # the timed loop cycles through `rotate` fields of the same recipe (other seeds): a step never
    # reads an input that earlier steps left in the Infinity Cache
    inputs = [d_in]
    for k in range(1, max(1, args.rotate)):
        f = make_field(seed + 1000 * k)
        inputs.append(f[slab.offset:slab.offset + n].clone() if sharded else f)
        del f
    cur = {"i": 0}
    d_out = torch.empty(n, dtype=tdt, device=dev)
    stream = torch.cuda.current_stream(dev)
    r = cz.Resource(cz.F4 if esz == 4 else cz.F8, my_dims, predictor, stream=stream.cuda_stream)
    hist = torch.empty(2 * 512 + 1, dtype=torch.int32, device=dev)  # counts + the overflow word
    mm = torch.empty(2, dtype=torch.float64, device=dev)
    nbytes_in = esz * n  # this rank's bytes
    total_bytes = esz * n_full * (world if weak else 1)
    state = {"scratch": None, "parts": None}

    def compress():
        x = inputs[cur["i"]]
        if not sharded:
            ptr, nb, _ = r.compress(x.data_ptr(), args.eb, mode)
            return ptr, nb
        # pass 1 -> histogram all-reduce (RCCL, ordered on this stream: no host sync) -> finish;
        # Rel mode: eb times the whole field's value range (one more all-reduce); a slab past its
        # outlier capacity makes every rank repeat together (shard.compress_fields_sharded)
        (ptr, nb), = shard.compress_fields_sharded([r], [x], args.eb, dist, mode=1 if mode == cz.Rel else 0,
                                                   device=dev, hists=hist.view(1, -1))
        return ptr, nb

    def step(acc=None, rot=True, gather=False):
        if acc is not None:  # phase split: nothing of the previous step is still queued
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        ptr, nb = compress()  # host-synchronous (the archive header is read back)
        t1 = time.perf_counter()
        # RCCL gather of the per-rank archives to the root: output collection, not part of the
        # timed compress+decompress (each rank's archive stays resident and is decompressed
        # there); timed in the phase pass and done before the root's checks
        if world > 1 and (gather or acc is not None):
            view, state["scratch"] = archive_view(ptr, nb, dev, state["scratch"])
            if args.backend == "gloo":  # (rehearsal: gloo moves host tensors)
                parts = shard.gather_to_root(view.cpu(), dist, 0)
                state["parts"] = None if parts is None else [q.to(dev) for q in parts]
            else:
                state["parts"] = shard.gather_to_root(view, dist, 0)
        t2 = time.perf_counter()
        r.decompress(ptr, nb, d_out.data_ptr())
        if acc is not None:
            torch.cuda.synchronize()
            acc[0] += t1 - t0
            acc[1] += t2 - t1
            acc[2] += time.perf_counter() - t2
        if rot:
            cur["i"] = (cur["i"] + 1) % len(inputs)
        return ptr, nb

    def barrier():
        if dist is not None:
            dist.barrier()

    r.enable_timing(False)
    err = 0.0
    for w in range(max(args.warmup, len(inputs))):
        x = inputs[cur["i"]]
        step()
        torch.cuda.synchronize()
        # correctness guard on the measured configuration (error bound, every element, every field)
        err = max(err, (d_out.double() - x.double()).abs().max().item())
    cur["i"] = 0
    eb_abs = r.header.rc.eb  # Rel mode: eb * value range
    # the reconstruction is computed in T (lrz_x.cuhip.inl / spline3.inl), so T's rounding at the
    # field's magnitude adds to the bound (f32 at |x| ~ 256, HACC-like config 3: ~8e-6)
    ulp = (2.0 ** -23 if esz == 4 else 2.0 ** -52) * max(x.abs().max().item() for x in inputs)
    assert err <= 1.001 * eb_abs + ulp, f"error bound violated: {err} > {eb_abs} (+ulp {ulp})"

    # timed region: the library's HIP-event stage timing is OFF (its event records would add
    # barrier packets to the stream); the per-stage/kernel durations come from a second pass.
    # Decompress is asynchronous: step i's decompress overlaps the host side of step i+1's
    # compress on the same stream (nothing is skipped: every step's kernels run in order).
    def timed(rot):
        cur["i"] = 0
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step(rot=rot)
        torch.cuda.synchronize()
        barrier()
        return time.perf_counter() - t0

    dt_same = timed(False)  # every step on the same field (its input may stay cached)
    dt = timed(True)        # `value`: the steps cycle through the distinct fields
    # host-clock phase split (a separate pass: each step starts and ends with an idle stream)
    acc = [0.0, 0.0, 0.0]
    for _ in range(args.steps):
        step(acc)
    cur["i"] = 0
    # same steps again with stage timing on (HIP events on the manager's stream)
    r.enable_timing(True)
    stage_acc = np.zeros(cz.T_COUNT)
    for _ in range(args.steps):
        ptr, nb = step()
        torch.cuda.synchronize()
        stage_acc += np.array(r.stage_times())
    r.enable_timing(False)
    cur["i"] = 0
    ptr, nb = step(rot=False, gather=True)  # field 0's archive for what follows (CR, merge, roofline)
    torch.cuda.synchronize()
    if dist is not None:
        t = torch.tensor([dt, dt_same, acc[0], acc[1], acc[2]], device=dev if args.backend == "nccl" else "cpu",
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt, dt_same, acc[0], acc[1], acc[2] = t.tolist()
    ms_per_step = 1e3 * dt / args.steps
    value = total_bytes * args.steps / dt / 1e9
    st = stage_acc / args.steps
    comp_ms, decomp_ms = st[cz.T_COMPRESS], st[cz.T_DECOMPRESS]

    # whole-field archive at the root: merge the gathered slabs (host), decompress it on the root
    merged_ok, arch_bytes_total = None, nb
    if sharded:
        parts = state["parts"]
        if rank == 0:
            host_parts = [p.cpu().numpy().tobytes() for p in parts]
            merged = shard.merge(host_parts, dims, [s.offset for s in shard.plan_slabs(dims, world)])
            arch_bytes_total = len(merged)
            hdr = cz.psz_header.from_buffer_copy(merged[:176])
            r_full = cz.Resource(cz.F4 if esz == 4 else cz.F8, dims, predictor, stream=stream.cuda_stream,
                                 header=hdr)
            d_arch = torch.frombuffer(bytearray(merged), dtype=torch.uint8).to(dev)
            out = torch.empty(n_full, dtype=tdt, device=dev)
            r_full.decompress(d_arch.data_ptr(), len(merged), out.data_ptr())
            torch.cuda.synchronize()
            e_full = (out.double() - d_full.double()).abs().max().item()
            merged_ok = bool(e_full <= 1.001 * eb_abs + ulp)
            r_full.close()
            del out, d_arch, d_full
        barrier()
    elif weak:
        # the root decompresses every rank's gathered archive against that rank's field (the
        # recipe is deterministic: regenerated from the rank's seed)
        parts = state["parts"]
        if rank == 0:
            ok = True
            for k, p in enumerate(parts):
                hdr = cz.psz_header.from_buffer_copy(p[:176].cpu().numpy().tobytes())
                rk = cz.Resource(cz.F4 if esz == 4 else cz.F8, dims, predictor, stream=stream.cuda_stream, header=hdr)
                out = torch.empty(n_full, dtype=tdt, device=dev)
                rk.decompress(p.data_ptr(), p.numel(), out.data_ptr())
                fk = make_field(seed - rank + k)
                torch.cuda.synchronize()
                e_k = (out.double() - fk.double()).abs().max().item()
                bound = 1.001 * hdr.rc.eb + ulp  # (the header's eb is absolute: Rel mode scaled it)
                ok = ok and e_k <= bound
                rk.close()
                del out, fk
            merged_ok = bool(ok)
            arch_bytes_total = sum(int(p.numel()) for p in parts)
        barrier()
    ratio = esz * n_full / arch_bytes_total if sharded else nbytes_in / nb

    # dominant kernel roofline (algorithmic bytes per launch / event-measured duration), rank 0
    ino = r.internals()
    splen = r.header.splen
    arch_bytes = nb
    pname = "spline3" if predictor == cz.Spline else "lorenzo"
    if ino.layout == cz.LAYOUT_BRICK:
        # fused brick path (brick.hip): pass 1 reads the field once and writes brick-ordered codes,
        # the per-brick u16 histograms and the outlier cells; pass 2 (+ the plan kernel) reads the
        # codes and writes the archive; decompress is one kernel (decode + reconstruct)
        nbricks = -(-n // (256 * 64))
        kernels = {
            "brick_scan": (st[cz.T_PREDICT], esz * n + 2 * n + 2 * 1024 * nbricks + 8 * splen,
                           ["k_brick3_scan", "k_brick1_scan"]),
            "brick_plan+pack": (st[cz.T_ENCODE], 2 * 1024 * nbricks + 2 * n + arch_bytes,
                                ["k_brick_plan", "k_brick3_pack"]),
            "brick_decode": (st[cz.T_DECODE] + st[cz.T_RECON], arch_bytes + esz * n,
                             ["k_brick3_decode", "k_brick1_decode"]),
        }
    else:
        kernels = {
            # predictor: read N*esz, write codes N*2 + outlier cells 8/each
            f"{pname}_c": (st[cz.T_PREDICT], esz * n + 2 * n + 8 * splen, [f"k_{pname}_c", "k_lorenzo_c"]),
            # encoder: read codes N*2, write bitstream (archive - metadata)
            "hf_encode": (st[cz.T_ENCODE], 2 * n + arch_bytes, ["k_hf_pack", "k_hf_gather", "k_hf_encode"]),
            # decoder: read bitstream, write codes N*2
            "hf_decode": (st[cz.T_DECODE], arch_bytes + 2 * n, ["k_hf_decode"]),
            # reconstruct: read codes N*2 (+ sparse outlier cells), write N*esz
            f"{pname}_x": (st[cz.T_RECON], 2 * n + esz * n, [f"k_{pname}_x", "k_lorenzo_x"]),
        }
    dom = max(kernels, key=lambda k: kernels[k][0])
    d_ms, d_bytes, _ = kernels[dom]
    achieved = d_bytes / (d_ms * 1e-3) / 1e9 if d_ms > 0 else None
    # HBM bytes per launch of the same kernel from the committed PMC summary of THIS config
    # (profiles/pmc_config<N>.json: rocprofv3 FETCH_SIZE/WRITE_SIZE passes, scripts/pmc_config.sh);
    # null when this config has not been profiled or the launch is a slab (N > 1)
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_config{args.config}.json")
    if os.path.exists(pmc_path) and not sharded:
        try:
            pmc = json.load(open(pmc_path))
            hits = [v["hbm_bytes_per_launch"] for k, v in pmc.items()
                    if any(k.startswith(p) for p in kernels[dom][2]) and "hbm_bytes_per_launch" in v]
            traffic = int(sum(hits)) if hits else None
        except Exception:
            traffic = None
    roofline = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1) if achieved else None,
                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                "traffic": traffic, "algorithmic_bytes": int(d_bytes)}

    # the other codebook modes (psz_amd_set_codebook), 3-D brick fields, beside the default line
    # (never `value`): EXACT = the reference's heap codebook built on the host (byte-identical
    # archives to the reference encoder's; its histogram goes to the host and the book comes back
    # behind a device-polled gate), STREAM = the sampled device codebook + one predict/pack pass
    other_modes = None
    if (world == 1 and not args.no_other_modes and ino.layout == cz.LAYOUT_BRICK and dims[1] > 1 and dims[2] > 1
            and predictor != cz.Spline):
        other_modes = {}
        for name, mode in (("exact", cz.CODEBOOK_EXACT), ("stream", cz.CODEBOOK_STREAM)):
            r.set_codebook(mode)
            cur["i"] = 0
            for _ in range(args.warmup):
                step(rot=False)
            torch.cuda.synchronize()
            e_s = (d_out.double() - d_in.double()).abs().max().item()
            ptr_s, nb_s = step(rot=False)
            dt_s = timed(True)
            r.enable_timing(True)
            st_s = np.zeros(cz.T_COUNT)
            for _ in range(args.steps):
                step()
                torch.cuda.synchronize()
                st_s += np.array(r.stage_times())
            r.enable_timing(False)
            st_s /= args.steps
            c_ms = st_s[cz.T_COMPRESS]
            other_modes[name] = {
                "value": round(total_bytes * args.steps / dt_s / 1e9, 2),
                "ms_per_step": round(1e3 * dt_s / args.steps, 4),
                "compress_ms": round(float(c_ms), 4),
                "compress_gbps": round(nbytes_in / (c_ms * 1e-3) / 1e9, 2) if c_ms > 0 else None,
                "compress_roofline_frac": round(nbytes_in / (c_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if c_ms > 0 else None,
                "stages_ms": {k: round(float(st_s[i]), 4) for k, i in
                              [("predict", cz.T_PREDICT), ("book", cz.T_BOOK), ("encode", cz.T_ENCODE),
                               ("finalize", cz.T_FINALIZE)]},
                "compression_ratio": round(nbytes_in / nb_s, 3),
                "cr_vs_default_pct": round(100.0 * ((nbytes_in / nb_s) / (nbytes_in / nb) - 1.0), 3),
                "max_abs_err": e_s}
            assert e_s <= 1.001 * eb_abs + ulp, f"codebook mode {name}: error bound violated: {e_s}"
        r.set_codebook(cz.CODEBOOK_SAMPLED)
        cur["i"] = 0
        ptr, nb = step(rot=False)  # the default archive again for what follows
        torch.cuda.synchronize()

    # end-to-end path from/to host memory (pinned), for DESIGN.md (never `value`)
    e2e = None
    if not args.no_e2e and not args.profile_only and world == 1:
        h_in = d_in.cpu().pin_memory()
        h_arch = torch.empty(nb, dtype=torch.uint8).pin_memory()
        h_out = torch.empty(n, dtype=tdt).pin_memory()
        d_arch = torch.empty(nb, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        reps = 3
        for _ in range(reps):
            d_in.copy_(h_in, non_blocking=True)
            ptr, nb2, _ = r.compress(d_in.data_ptr(), args.eb, mode)
            cz.hip_memcpy(h_arch.data_ptr(), ptr, nb2, 2)
            d_arch[:nb2].copy_(h_arch[:nb2], non_blocking=True)
            r.decompress(d_arch.data_ptr(), nb2, d_out.data_ptr())
            h_out.copy_(d_out, non_blocking=True)
            torch.cuda.synchronize()
        e2e = round(nbytes_in * reps / (time.perf_counter() - t1) / 1e9, 2)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_only:
        if predictor == cz.Spline:
            cpu = {"value": None, "unit": "GB/s", "cores": 0, "kind": "reference",
                   "reason": "the reference has no CPU spline path (spline3.inl is CUDA-only, SURVEY.md §0.5)"}
        elif esz == 4:
            cpu = cpu_baseline(d_in, dims, args.eb, nbytes_in)

    if rank == 0:
        tg_ms = 1e3 * acc[1] / args.steps
        tc_ms = 1e3 * acc[0] / args.steps
        td_ms = 1e3 * acc[2] / args.steps
        line = {
            "metric": METRICS[args.config],
            # only config 2 is BASELINE.json's metric workload; the others use the same fields
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if sharded or (world == 1 and args.scaling == "strong") else "weak",
            "vs_baseline": None,
            "dtype": "f64" if esz == 8 else "f32",
            "data": f"synthetic (SURVEY.md §8d config-{args.config} recipe" + (", seed per rank)" if weak else ")"),
            "config": {"workload": f"config{args.config}: {dims[0]}x{dims[1]}x{dims[2]} "
                                   f"{'f64' if esz == 8 else 'f32'}, {'rel' if mode == cz.Rel else 'abs'} "
                                   f"eb={args.eb}, {'spline3' if predictor == cz.Spline else 'Lorenzo'} + "
                                   "histogram + Huffman, compress+decompress per step",
                       "field_bytes": esz * n_full, "per_rank_bytes": nbytes_in,
                       "parallelism": (f"dp{world} (tile-aligned z-slabs of one field: histogram all-reduce; "
                                       "archive gather to rank 0 outside the timed steps)") if sharded else
                                      (f"dp{world} (an independent field per rank, no collective in the timed "
                                       "steps; archives gathered to rank 0 outside them)" if weak else "single GPU")},
            "compress_gbps": round(nbytes_in / (comp_ms * 1e-3) / 1e9, 2) if comp_ms > 0 else None,
            "decompress_gbps": round(nbytes_in / (decomp_ms * 1e-3) / 1e9, 2) if decomp_ms > 0 else None,
            "compress_roofline_frac": round(nbytes_in / (comp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if comp_ms > 0 else None,
            "decompress_roofline_frac": round(nbytes_in / (decomp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if decomp_ms > 0 else None,
            "rotating_inputs": len(inputs),
            "same_field_value": round(total_bytes * args.steps / dt_same / 1e9, 2),
            "same_field_ms_per_step": round(1e3 * dt_same / args.steps, 4),
            # host clock, a separate pass in which every step starts and ends on an idle stream
            "host_phases_ms": {"compress_call": round(tc_ms, 4), "gather": round(tg_ms, 4),
                               "decompress_to_idle": round(td_ms, 4)},
            "field_compress_call_gbps": round(total_bytes / (tc_ms * 1e-3) / 1e9, 2) if tc_ms > 0 else None,
            "field_compress_gather_gbps": round(total_bytes / ((tc_ms + tg_ms) * 1e-3) / 1e9, 2) if tc_ms > 0 else None,
            "value_incl_gather": (round(total_bytes / ((ms_per_step + tg_ms) * 1e-3) / 1e9, 2) if world > 1 else None),
            "compression_ratio": round(ratio, 3),
            "stages_ms": {k: round(float(st[i]), 4) for k, i in
                          [("predict", cz.T_PREDICT), ("book", cz.T_BOOK), ("encode", cz.T_ENCODE),
                           ("finalize", cz.T_FINALIZE), ("compress", cz.T_COMPRESS),
                           ("scatter", cz.T_SCATTER), ("decode", cz.T_DECODE), ("recon", cz.T_RECON),
                           ("decompress", cz.T_DECOMPRESS)]},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "e2e_host_gbps": e2e,
            "codebook": ("device two-queue book of the full histogram" if predictor == cz.Spline or sharded
                         else "two-queue book of pass 1's brick sample + 1 (host, mid-pass)"
                         if ino.layout == cz.LAYOUT_BRICK and (dims[2] > 1 or dims[1] == 1)
                         else "reference heap book of the full histogram (host)"),
            # `value` is measured with the default (SAMPLED) codebook mode: unless the line above
            # names the reference heap book, the archive's Huffman book is NOT the reference
            # encoder's (same quantization codes and decompressed field, different bitstream);
            # the EXACT mode's reference-identical archive is timed beside it
            "archive_reference_identical": bool(
                predictor != cz.Spline and not sharded and not (ino.layout == cz.LAYOUT_BRICK and (dims[2] > 1 or dims[1] == 1))),
            "value_exact_codebook": (other_modes or {}).get("exact", {}).get("value"),
            "other_codebook_modes": other_modes,
            "max_abs_err": err,
        }
        if sharded:
            line["merged_archive_bytes"] = arch_bytes_total
            line["merged_decompress_ok"] = merged_ok
        elif weak:
            line["gathered_archive_bytes"] = arch_bytes_total
            line["gathered_decompress_ok"] = merged_ok
        print(json.dumps(line), flush=True)
    r.close()


def host_cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def cpu_baseline(d_in, dims, eb, nbytes_in):
    """The reference CPU path (psz_seq_core: lrz.seq.cc, hist_generic.seq.cc, hf_bk*.seq.cc,
    compiled from the reference's own sources into oracle/_ref by oracle/Makefile; that .so
    travels to the GPU box with the tree) on the same field, this host:
      * 1 thread (the reference is single-threaded): c_lorenzo + histogram + codebook (compress;
        the reference has no CPU Huffman encoder) and x_lorenzo (decompress; no CPU decoder);
      * all cores, parallelised by us: the same reference calls on tile-aligned slabs (z: 8-plane,
        2-D: 32-row, 1-D: 1024-element multiples; tile-independent), one thread each (ctypes
        drops the GIL), wall time of the slowest + one codebook.
    Null if oracle/_ref is absent."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import pyoracle
    except Exception:
        return None
    if not pyoracle.ref_available():
        return None

    from cusz_amd.shard import plan_slabs, tile_extent

    host = d_in.cpu().numpy()
    aff = sorted(os.sched_getaffinity(0))
    t = pyoracle.ref_time_stages(host, dims, eb)
    total_ms = t["c_lorenzo"] + t["histogram"] + t["codebook"] + t["x_lorenzo"]
    # all-core variant: slabs along the slowest axis over min(cores, 16) threads (the GPU box
    # grants 16 CPUs per GPU), at most one slab per tile row
    axis, tl = tile_extent(dims)
    nth = max(1, min(len(aff), 16, (dims[axis] + tl - 1) // tl))
    slabs = [sl for sl in plan_slabs(dims, nth) if sl.count]
    # every slab runs the same timed reference stages as the 1-thread leg, one thread per slab in
    # the shim, buffers allocated before a barrier that starts all stage clocks together; the
    # parallel time is the slowest thread's stage sum, plus one codebook
    ts, _wall = pyoracle.ref_time_stages_par(host, [(sl.offset, sl.dims) for sl in slabs], eb)
    par_ms = max(u["c_lorenzo"] + u["histogram"] + u["x_lorenzo"] for u in ts) + t["codebook"]
    return {"value": round(nbytes_in / (total_ms * 1e-3) / 1e9, 4), "unit": "GB/s", "cores": 1,
            "kind": "reference", "host_cpu": host_cpu_model(),
            "sample": f"full {dims[0]}x{dims[1]}x{dims[2]} f32 field; reference CPU path "
                      f"(lrz.seq.cc c_lorenzo {t['c_lorenzo']:.0f} ms + hist {t['histogram']:.0f} ms + "
                      f"codebook {t['codebook']:.2f} ms + x_lorenzo {t['x_lorenzo']:.0f} ms; "
                      "no CPU Huffman in the reference)",
            "all_cores": {"value": round(nbytes_in / (par_ms * 1e-3) / 1e9, 4), "cores": len(slabs),
                          "kind": "reference, parallelised by us over tile-aligned slabs",
                          "timing": "slowest thread's c_lorenzo + hist + x_lorenzo, threads started together after their allocations, + codebook"}}


def bench_sharded(args, world, rank, dist, dev):
    """config 4: six Nyx-like 512^3 f32 fields, each split into tile-aligned z-slabs, slab r of
    every field on rank r.  One step = sharded compress of all six fields with one codebook per
    field (value ranges by the library's extrema kernel + one all-reduce, pass 1 per slab, ONE
    all-reduce of the [6, 1024] histograms, finish per slab), then the gather of every rank's six
    archives to rank 0.  value = 6 x 512 MiB / compress time (max over ranks); the
    compress+gather time is reported beside it."""
    import torch

    import cusz_amd as cz
    from cusz_amd import datagen, shard

    full = (512, 512, 512)
    # abs 1e-4: the 200 G velocity fields put most elements outside radius 512,
    # past the reference's 10 % outlier cap; the capacity grows (the first step repeats once per
    # manager, during warmup).  --rel: value-range relative bound instead
    eb = args.eb if args.eb is not None else 1e-4
    mode4 = cz.Rel if args.rel else cz.Abs
    sl = shard.plan_slabs(full, world)[rank]
    z0 = sl.offset // (full[0] * full[1])
    fields = datagen.nyx_fields_torch(full, device=dev, z0=z0, z1=z0 + sl.dims[2])
    stream = torch.cuda.current_stream(dev)
    res = [cz.Resource(cz.F4, sl.dims, stream=stream.cuda_stream) for _ in fields]
    hists = torch.empty((len(fields), 1026), dtype=torch.int32, device=dev)
    total_bytes = 6 * full[0] * full[1] * full[2] * 4
    state = {"scratch": None}

    def compress():
        return shard.compress_fields_sharded(res, fields, eb, dist, mode=mode4, device=dev, hists=hists)

    def gather(arch):
        sizes = [nb for _, nb in arch]
        if state["scratch"] is None or state["scratch"].numel() < sum(sizes):
            state["scratch"] = torch.empty(sum(sizes), dtype=torch.uint8, device=dev)
        buf = state["scratch"][:sum(sizes)]
        off = 0
        for (p, nb) in arch:
            cz.hip_memcpy(buf.data_ptr() + off, p, nb, 3)
            off += nb
        meta = torch.tensor(sizes, dtype=torch.int64, device=dev)
        if dist is None:
            return [buf], [meta.view(torch.uint8)]
        return shard.gather_to_root(buf, dist, 0), shard.gather_to_root(meta.view(torch.uint8), dist, 0)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        gather(compress())
    torch.cuda.synchronize(dev)
    barrier()
    tc = tg = 0.0
    for _ in range(args.steps):
        t0 = time.perf_counter()
        arch = compress()  # host-synchronous (every slab's header is read back)
        t1 = time.perf_counter()
        got = gather(arch)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        tc += t1 - t0
        tg += t2 - t1
    barrier()
    if dist is not None:
        t = torch.tensor([tc, tc + tg], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        tc, tcg = t.tolist()
    else:
        tcg = tc + tg
    # validation on the root: merge the slabs of field 0 (density) and field 1 (a velocity: most
    # elements outliers at abs 1e-4) and decompress the merged archives
    merged_ok, merged_len = None, None
    if rank == 0:
        bufs, metas = got
        oks = []
        for fi in (0, 1):
            parts = []
            for b, m in zip(bufs, metas):
                sizes = m.view(torch.int64).tolist()
                off = sum(sizes[:fi])
                parts.append(b[off:off + sizes[fi]].cpu().numpy().tobytes())
            merged = shard.merge(parts, full)
            if fi == 0:
                merged_len = len(merged)
            if world == 1:
                hdr = cz.psz_header.from_buffer_copy(merged[:176])  # the archive's header, as the CLI does
                r_full = cz.Resource(cz.F4, full, stream=stream.cuda_stream, header=hdr)
                d_arch = torch.frombuffer(bytearray(merged), dtype=torch.uint8).to(dev)
                out = torch.empty(fields[fi].numel(), dtype=torch.float32, device=dev)
                r_full.decompress(d_arch.data_ptr(), len(merged), out.data_ptr())
                torch.cuda.synchronize(dev)
                ulp = 2.0 ** -23 * fields[fi].abs().max().item()
                eb0 = eb * (fields[fi].max() - fields[fi].min()).item() if args.rel else eb
                oks.append(bool((out - fields[fi]).abs().max().item() <= 1.001 * eb0 + ulp))
                r_full.close()
                del d_arch, out
        merged_ok = all(oks) if oks else None
        line = {
            "metric": METRICS[4], "value": round(total_bytes * args.steps / tc / 1e9, 2), "unit": "GB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * tc / args.steps, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (SURVEY.md §8d config-4 recipe)",
            "config": {"workload": f"config4: 6 Nyx-like 512x512x512 f32 fields, {'rel' if args.rel else 'abs'} eb={eb}, z-slabs "
                                   f"{sl.dims[2]} planes per rank, global codebook per field",
                       "parallelism": f"dp{world} (z-slabs, 2 all-reduces + gather to root)"},
            "compress_gather_ms_per_step": round(1e3 * tcg / args.steps, 4),
            "compress_gather_gbps": round(total_bytes * args.steps / tcg / 1e9, 2),
            "merged_field0_bytes": merged_len, "merged_fields01_decompress_ok": merged_ok,
            "archive_bytes_per_step": int(sum(nb for _, nb in arch)),
        }
        print(json.dumps(line), flush=True)
    for r in res:
        r.close()


if __name__ == "__main__":
    sys.exit(main())
