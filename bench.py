#!/usr/bin/env python3
"""bench.py -- device-resident compress+decompress throughput of cusz_amd on MI355X.

Metric (BASELINE.json): "device-resident compress+decompress GB/s (input bytes),
512^3 f32 abs eb=1e-4".  One step = psz_compress_float + psz_decompress_float of one
512^3 f32 field already resident in HBM (config 2 of BASELINE.json: Lorenzo-3D + histogram
+ Huffman), through the C-ABI.  value = (bytes of input processed by all ranks) / time.

Multi-GPU (torchrun, one rank per GPU): every rank compresses and decompresses its own
512^3 field (the path shards by independent fields / tile-aligned slabs, no data-path
collective) -> "scaling": "weak"; barrier + synchronize bracket the timed steps and the
max time over ranks is used.

Extra fields on the JSON line:
  roofline      dominant kernel: algorithmic bytes / its HIP-event duration vs 8 TB/s
  cpu_baseline  the reference's own CPU path (compiled from /root/reference into
                oracle/_ref; single thread) timed on this host on the same 512^3 field
  stages_ms     per-stage device times of the last step (HIP events in the library)
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
    4: "aggregate sharded compress GB/s (input bytes), Nyx-like 6x512³ f32 r2r eb=1e-4, z-slabs per rank",
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
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the host-memory (PCIe) path timing")
    ap.add_argument("--profile-only", action="store_true", help="few steps, no baselines (rocprof)")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch

    import cusz_amd as cz
    from cusz_amd import datagen

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist

        torch.cuda.set_device(local)
        tdist.init_process_group("nccl")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.config == 4:
        return bench_sharded(args, world, rank, dist, dev)

    cfg = {1: ("3600x1800", 1e-4, cz.Abs, cz.Lorenzo, torch.float32),
           2: ("512x512x512", 1e-4, cz.Abs, cz.Lorenzo, torch.float32),
           3: ("280953867", 1e-4, cz.Abs, cz.Lorenzo, torch.float32),
           5: ("512x512x512", 1e-6, cz.Rel, cz.Spline, torch.float64)}[args.config]
    dims = tuple(int(v) for v in (args.dims or cfg[0]).lower().split("x"))
    dims = (dims + (1, 1))[:3]
    args.eb = args.eb if args.eb is not None else cfg[1]
    mode, predictor, tdt = cfg[2], cfg[3], cfg[4]
    esz = 8 if tdt == torch.float64 else 4
    n = dims[0] * dims[1] * dims[2]
    nbytes_in = esz * n

    if args.config == 1:
        d_in = torch.from_numpy(datagen.cesm2d_np(dims[:2], seed=1 + rank)).to(dev)
    elif args.config == 3:
        d_in = datagen.hacc1d_torch(n, seed=3 + rank, device=dev)
    else:
        d_in = datagen.smooth3d_torch(dims, seed=(5 if args.config == 5 else 2) + rank, dtype=tdt, device=dev)
    d_out = torch.empty(n, dtype=tdt, device=dev)
    stream = torch.cuda.current_stream(dev)
    r = cz.Resource(cz.F4 if esz == 4 else cz.F8, dims, predictor, stream=stream.cuda_stream)
    r.enable_timing(True)

    def barrier():
        if dist:
            tdist.barrier()

    def step():
        ptr, nb, _ = r.compress(d_in.data_ptr(), args.eb, mode)
        r.decompress(ptr, nb, d_out.data_ptr())
        return ptr, nb

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # correctness guard on the measured configuration (error bound, every element)
    err = (d_out.double() - d_in.double()).abs().max().item()
    eb_abs = r.header.rc.eb  # Rel mode: eb * value range
    # the reconstruction is computed in T (lrz_x.cuhip.inl / spline3.inl), so T's rounding at the
    # field's magnitude adds to the bound (f32 at |x| ~ 256, HACC-like config 3: ~8e-6)
    ulp = (2.0 ** -23 if esz == 4 else 2.0 ** -52) * d_in.abs().max().item()
    assert err <= 1.001 * eb_abs + ulp, f"error bound violated: {err} > {eb_abs} (+ulp {ulp})"

    # timed region: the library's HIP-event stage timing is OFF (its event records would add
    # barrier packets to the stream); the per-stage/kernel durations come from a second pass
    r.enable_timing(False)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ptr, nb = step()
        torch.cuda.synchronize()  # decompress is asynchronous; close the step
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    # same steps again with stage timing on (HIP events on the manager's stream)
    r.enable_timing(True)
    stage_acc = np.zeros(cz.T_COUNT)
    for _ in range(args.steps):
        ptr, nb = step()
        torch.cuda.synchronize()
        stage_acc += np.array(r.stage_times())
    if dist:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        dt = t.item()
    ms_per_step = 1e3 * dt / args.steps
    value = world * nbytes_in * args.steps / dt / 1e9
    st = stage_acc / args.steps
    comp_ms, decomp_ms = st[cz.T_COMPRESS], st[cz.T_DECOMPRESS]
    ratio = nbytes_in / nb

    # dominant kernel roofline (algorithmic bytes per launch / event-measured duration)
    ino = r.internals()
    splen = r.header.splen
    arch_bytes = nb
    pname = "spline3" if predictor == cz.Spline else "lorenzo"
    if ino.layout == cz.LAYOUT_BRICK:
        # fused brick path (brick.hip): pass 1 reads the field once and writes brick-ordered codes,
        # the per-brick u16 histograms and the outlier cells; pass 2 (+ the plan kernel) reads the
        # codes and writes the archive; decompress is one kernel (decode + reconstruct)
        nbricks = n // (256 * 64)
        kernels = {
            "brick_scan": (st[cz.T_PREDICT], esz * n + 2 * n + 2 * 1024 * nbricks + 8 * splen, ["k_brick3_scan"]),
            "brick_plan+pack": (st[cz.T_ENCODE], 2 * 1024 * nbricks + 2 * n + arch_bytes,
                                ["k_brick_plan", "k_brick3_pack"]),
            "brick_decode": (st[cz.T_DECODE] + st[cz.T_RECON], arch_bytes + esz * n, ["k_brick3_decode"]),
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
    # null when this config has not been profiled
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", f"pmc_config{args.config}.json")
    if os.path.exists(pmc_path):
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

    # end-to-end path from/to host memory (pinned), for DESIGN.md (never `value`)
    e2e = None
    if not args.no_e2e and not args.profile_only and rank == 0:
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
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not args.profile_only and esz == 4 \
            and predictor == cz.Lorenzo:
        cpu = cpu_baseline(d_in, dims, args.eb, nbytes_in)

    if rank == 0:
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if esz == 8 else "f32",
            "data": f"synthetic (SURVEY.md §8d config-{args.config} recipe, seed per rank)",
            "config": {"workload": f"config{args.config}: {dims[0]}x{dims[1]}x{dims[2]} "
                                   f"{'f64' if esz == 8 else 'f32'}, {'rel' if mode == cz.Rel else 'abs'} "
                                   f"eb={args.eb}, {'spline3' if predictor == cz.Spline else 'Lorenzo'} + "
                                   "histogram + Huffman, compress+decompress per step",
                       "per_rank_field_bytes": nbytes_in, "parallelism": f"dp{world} (independent fields)"},
            "compress_gbps": round(nbytes_in / (comp_ms * 1e-3) / 1e9, 2) if comp_ms > 0 else None,
            "decompress_gbps": round(nbytes_in / (decomp_ms * 1e-3) / 1e9, 2) if decomp_ms > 0 else None,
            "compress_roofline_frac": round(nbytes_in / (comp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if comp_ms > 0 else None,
            "decompress_roofline_frac": round(nbytes_in / (decomp_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if decomp_ms > 0 else None,
            "compression_ratio": round(ratio, 3),
            "stages_ms": {k: round(float(st[i]), 4) for k, i in
                          [("predict", cz.T_PREDICT), ("book", cz.T_BOOK), ("encode", cz.T_ENCODE),
                           ("finalize", cz.T_FINALIZE), ("compress", cz.T_COMPRESS),
                           ("scatter", cz.T_SCATTER), ("decode", cz.T_DECODE), ("recon", cz.T_RECON),
                           ("decompress", cz.T_DECOMPRESS)]},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "e2e_host_gbps": e2e,
            "max_abs_err": err,
        }
        print(json.dumps(line), flush=True)
    r.close()
    if dist:
        tdist.destroy_process_group()


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
      * all cores, parallelised by us: the same reference calls on z-slabs of 8-plane multiples
        (tile-independent), one thread each (ctypes drops the GIL), wall time of the slowest +
        one codebook.
    Null if oracle/_ref is absent."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    try:
        import pyoracle
    except Exception:
        return None
    if not pyoracle.ref_available():
        return None
    import concurrent.futures as cf

    host = d_in.cpu().numpy()
    aff = sorted(os.sched_getaffinity(0))
    t = pyoracle.ref_time_stages(host, dims, eb)
    total_ms = t["c_lorenzo"] + t["histogram"] + t["codebook"] + t["x_lorenzo"]
    # all-core variant: z-slabs over min(cores, 16) threads (the GPU box grants 16 CPUs per GPU)
    nth = max(1, min(len(aff), 16, dims[2] // 8))
    from cusz_amd.shard import plan_slabs

    slabs = [sl for sl in plan_slabs(dims, nth) if sl.count]
    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(len(slabs)) as ex:
        list(ex.map(lambda sl: pyoracle.ref_time_stages(host[sl.offset:sl.offset + sl.count], sl.dims, eb), slabs))
    par_ms = (time.perf_counter() - t0) * 1e3 + t["codebook"]
    return {"value": round(nbytes_in / (total_ms * 1e-3) / 1e9, 4), "unit": "GB/s", "cores": 1,
            "kind": "reference", "host_cpu": host_cpu_model(),
            "sample": f"full {dims[0]}x{dims[1]}x{dims[2]} f32 field; reference CPU path "
                      f"(lrz.seq.cc c_lorenzo {t['c_lorenzo']:.0f} ms + hist {t['histogram']:.0f} ms + "
                      f"codebook {t['codebook']:.2f} ms + x_lorenzo {t['x_lorenzo']:.0f} ms; "
                      "no CPU Huffman in the reference)",
            "all_cores": {"value": round(nbytes_in / (par_ms * 1e-3) / 1e9, 4), "cores": len(slabs),
                          "kind": "reference, parallelised by us over z-slabs"}}


def bench_sharded(args, world, rank, dist, dev):
    """config 4: six Nyx-like 512^3 f32 fields, each split into tile-aligned z-slabs, slab r of
    every field on rank r.  One step = sharded compress of all six fields with one codebook per
    field (pass 1 per slab, ONE all-reduce of the [6, 1024] histograms, finish per slab), then
    the gather of every rank's six archives to rank 0.  value = 6 x 512 MiB / compress time
    (max over ranks); the compress+gather time is reported beside it."""
    import numpy as np
    import torch

    import cusz_amd as cz
    from cusz_amd import datagen, shard

    if dist is None or not world > 1:
        import torch.distributed as tdist

        if not tdist.is_initialized():
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(29400 + os.getpid() % 1000))
            tdist.init_process_group("nccl", rank=0, world_size=1)
    import torch.distributed as tdist

    full = (512, 512, 512)
    # r2r 1e-4 (value-range relative): at abs 1e-4 the 200 G velocity fields put
    # far more than the 10 % outlier cap outside radius 512 (PSZ_WARN_OUTLIER_TOO_MANY)
    eb = args.eb if args.eb is not None else 1e-4
    sl = shard.plan_slabs(full, world)[rank]
    z0 = sl.offset // (full[0] * full[1])
    fields = datagen.nyx_fields_torch(full, device=dev, z0=z0, z1=z0 + sl.dims[2])
    stream = torch.cuda.current_stream(dev)
    res = [cz.Resource(cz.F4, sl.dims, stream=stream.cuda_stream) for _ in fields]
    for r in res:
        r.enable_timing(True)
    total_bytes = 6 * full[0] * full[1] * full[2] * 4

    def compress():
        return shard.compress_fields_sharded(res, fields, eb, tdist, mode=cz.Rel, device=dev)

    def gather(arch):
        sizes = [nb for _, nb in arch]
        buf = torch.empty(sum(sizes), dtype=torch.uint8, device=dev)
        off = 0
        for (p, nb) in arch:
            cz.hip_memcpy(buf.data_ptr() + off, p, nb, 3)
            off += nb
        meta = torch.tensor(sizes, dtype=torch.int64, device=dev)
        return shard.gather_to_root(buf, tdist, 0), shard.gather_to_root(meta.view(torch.uint8), tdist, 0)

    for _ in range(args.warmup):
        gather(compress())
    torch.cuda.synchronize(dev)
    tdist.barrier()
    tc = tg = 0.0
    for _ in range(args.steps):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        arch = compress()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        got = gather(arch)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        tc += t1 - t0
        tg += t2 - t1
    tdist.barrier()
    t = torch.tensor([tc, tc + tg], device=dev, dtype=torch.float64)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    tc, tcg = t.tolist()
    # validation on the root: merge the slabs of field 0 and decompress the merged archive
    merged_ok = None
    if rank == 0:
        bufs, metas = got
        parts = []
        for b, m in zip(bufs, metas):
            sizes = m.view(torch.int64).tolist()
            parts.append(b[: sizes[0]].cpu().numpy().tobytes())
        merged = shard.merge(parts, full)
        if world == 1:
            hdr = cz.psz_header.from_buffer_copy(merged[:176])  # the archive's header, as the CLI does
            r_full = cz.Resource(cz.F4, full, stream=stream.cuda_stream, header=hdr)
            d_arch = torch.frombuffer(bytearray(merged), dtype=torch.uint8).to(dev)
            out = torch.empty(fields[0].numel(), dtype=torch.float32, device=dev)
            r_full.decompress(d_arch.data_ptr(), len(merged), out.data_ptr())
            torch.cuda.synchronize(dev)
            ulp = 2.0 ** -23 * fields[0].abs().max().item()
            eb0 = eb * (fields[0].max() - fields[0].min()).item()
            merged_ok = bool((out - fields[0]).abs().max().item() <= 1.001 * eb0 + ulp)
            r_full.close()
        line = {
            "metric": METRICS[4], "value": round(total_bytes * args.steps / tc / 1e9, 2), "unit": "GB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * tc / args.steps, 4), "higher_is_better": True, "scaling": "strong",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (SURVEY.md §8d config-4 recipe)",
            "config": {"workload": f"config4: 6 Nyx-like 512x512x512 f32 fields, r2r eb={eb}, z-slabs "
                                   f"{sl.dims[2]} planes per rank, global codebook per field",
                       "parallelism": f"dp{world} (z-slabs, 1 all-reduce + gather to root)"},
            "compress_gather_ms_per_step": round(1e3 * tcg / args.steps, 4),
            "compress_gather_gbps": round(total_bytes * args.steps / tcg / 1e9, 2),
            "merged_field0_bytes": len(merged), "merged_field0_decompress_ok": merged_ok,
        }
        print(json.dumps(line), flush=True)
    for r in res:
        r.close()
    tdist.destroy_process_group()


if __name__ == "__main__":
    main()
