#!/usr/bin/env python3
"""bench.py -- the lzbench hot path on MI355X: lz4 -b64 over 1 GiB of synthetic text per GPU.

One step = one lzbench pass over the whole input (reference _lzbench/lzbench.cpp:384-393 and
:418-427): compress every 64 KiB chunk (HIP codec kernel, then size scan + packing with the
raw-store rule), then decompress every chunk from the packed stream.  Inputs are resident in
HBM when the timed region starts.  value = comp+decomp MB/s (MB = 1e6 B, lzbench.cpp:104-106)
= bytes processed by all ranks / (max over ranks of the timed wall time).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one
process per GPU, each compresses its own 1 GiB shard of independent chunks (weak scaling,
no data-path collective; the only cross-rank traffic is the barrier and the max-time
reduction on the control plane).

Also reported: the roofline of the dominant kernel (the LZ4 compress kernel, HIP events on
the stream it runs on), and the reference CPU codec (oracle/_ref, lz4 1.9.3 built from the
reference sources) timed on this host on a bounded sample of the same input (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
METRIC = "comp+decomp MB/s, lz4 -b64 on 1 GiB; ratio + bit-exact vs CPU ref"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(sample: np.ndarray, codec: str, chunk: int, level: int, iters: int, threads: int):
    """lzbench semantics on the host: best-of-iters compress pass + best-of-iters decompress
    pass over the sample (lzbench.cpp:379-469, -p1 fastest). Uses the reference build when
    present (kind 'reference'), else the repo's C restatement (kind 'port')."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    use_ref = O.have_ref()
    n = len(sample)
    best_c = best_d = float("inf")
    packed = cs = None
    for _ in range(iters):
        t = time.perf_counter()
        packed, cs = O.compress_chunks(sample, codec, chunk, level, use_ref=use_ref, threads=threads)
        best_c = min(best_c, time.perf_counter() - t)
    for _ in range(iters):
        t = time.perf_counter()
        r, out = O.decompress_chunks(packed, cs, n, codec, chunk, use_ref=use_ref, threads=threads)
        best_d = min(best_d, time.perf_counter() - t)
    ok = r == n and bool((out == sample).all())
    return {
        "value": round(n / (best_c + best_d) / 1e6, 2),
        "unit": "MB/s",
        "cores": max(threads, 1),
        "kind": "reference" if use_ref else "port",
        "sample": f"first {n >> 20} MiB of the same corpus, -b{chunk >> 10}, best of {iters} compress + {iters} "
                  f"decompress passes ({'lz4 1.9.3/snappy 1.1.8 compiled from the reference sources' if use_ref else 'oracle C restatement'})",
        "comp_MBps": round(n / best_c / 1e6, 2),
        "decomp_MBps": round(n / best_d / 1e6, 2),
        "roundtrip_ok": ok,
    }, packed, cs


def traffic_for(kernel):
    """HBM-side bytes per dispatch of `kernel` from the committed PMC profile (profiles/traffic.json,
    written by tools/pmc_traffic.sh: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes on the
    same workload), or None when no profile covers this kernel/workload."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            k = json.load(f)["kernels"].get(kernel)
        return None if k is None else int(k["traffic_bytes_per_dispatch"])
    except (OSError, KeyError, ValueError):
        return None


def kernel_name(codec):
    """Compressor kernel the C-ABI launches for `codec` (api.cpp lzh_compress_kernel_only)."""
    return "lzh_snappy_compress_v2_kernel" if codec == "snappy" else "lzh_lz4_compress_v2_kernel"


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--codec", default="lz4", choices=["lz4", "lz4fast", "snappy"])
    ap.add_argument("--level", type=int, default=1, help="lz4fast acceleration")
    ap.add_argument("--chunk-kib", type=int, default=64)
    ap.add_argument("--size-mib", type=int, default=1024, help="input bytes per GPU")
    ap.add_argument("--corpus", default="text", choices=["text", "json", "mixed", "random", "binary"])
    ap.add_argument("--cpu-sample-mib", type=int, default=256)
    ap.add_argument("--cpu-iters", type=int, default=3)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = 1 thread (lzbench semantics)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--backend", default="gloo", help="control-plane process group (no data-path collective)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))   # (ranks > GPUs only in rehearsal runs)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group(backend=args.backend)

    import lzbench_amd as L

    n = args.size_mib << 20
    chunk = args.chunk_kib << 10
    t = time.perf_counter()
    host = L.datagen(args.corpus, n, seed=12345 + rank)
    log(f"[rank {rank}] generated {n >> 20} MiB {args.corpus} in {time.perf_counter() - t:.1f}s")
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
    d_in[:n].copy_(torch.from_numpy(host))
    codec = L.DeviceCodec(args.codec, n, chunk, level=args.level)
    stream = torch.cuda.current_stream()

    nsteps = args.warmup + args.steps
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(nsteps)]

    def step(i):
        e = ev[i]
        e[0].record(stream)
        codec.compress_kernel_only(d_in)         # dominant kernel (roofline)
        e[1].record(stream)
        codec.compress_finish(d_in)              # size scan + packing (raw-store rule)
        e[2].record(stream)
        codec.decompress()                       # decode from the packed stream
        e[3].record(stream)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.warmup, nsteps):
        step(i)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())

    timed = ev[args.warmup:]
    k_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in timed]))
    f_ms = float(np.mean([e[1].elapsed_time(e[2]) for e in timed]))
    d_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in timed]))
    comp_total = codec.packed_total()
    roundtrip_ok = bool(torch.equal(codec.out[:n], d_in[:n])) and bool((codec.status >= 0).all().item())
    ratio = comp_total / n

    # bit-exactness vs the CPU reference on a sample: the packed prefix of the first m chunks
    # must equal the reference chunk loop's output for those chunks, sizes included
    result_extra = {}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        m = min(args.cpu_sample_mib << 20, n) // chunk * chunk or n
        sample = host[:m]
        cpu, ref_packed, ref_cs = cpu_baseline(sample, args.codec, chunk, args.level, args.cpu_iters,
                                               args.cpu_threads)
        if args.cpu_threads == 0:
            cpu_mt, _, _ = cpu_baseline(sample, args.codec, chunk, args.level, 1, min(16, os.cpu_count() or 1))
            result_extra["cpu_baseline_all_cores"] = cpu_mt
        gcs = codec.csizes[: len(ref_cs)].cpu().numpy().astype(np.uint64)
        gpk = codec.packed[: len(ref_packed)].cpu().numpy()
        result_extra["bit_exact_sample"] = bool((gcs == ref_cs).all() and (gpk == ref_packed).all())
        result_extra["bit_exact_sample_bytes"] = int(m)

    algo_bytes = n + comp_total                      # compress reads N, writes C
    achieved = algo_bytes / (k_ms * 1e-3) / 1e9
    dec_achieved = algo_bytes / (d_ms * 1e-3) / 1e9   # decompress reads C, writes N
    default_workload = args.codec == "lz4" and args.chunk_kib == 64 and args.corpus == "text" and args.size_mib == 1024
    total_bytes = world * n * args.steps
    value = total_bytes / elapsed / 1e6
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "MB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": f"synthetic {args.corpus} corpus (SURVEY.md 8(d) stand-in; enwik8/Silesia unavailable offline), "
                f"generated per rank, resident in HBM",
        "config": {
            "workload": f"{args.codec} -b{args.chunk_kib} on {n >> 20} MiB {args.corpus} per GPU, comp+decomp pass",
            "codec": args.codec,
            "chunk_kib": args.chunk_kib,
            "bytes_per_gpu": n,
            "chunks_per_gpu": int(codec.k),
            "parallelism": f"chunk-sharded x{world} (independent shards, no collective)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic_for(kernel_name(args.codec)) if default_workload else None,
            "traffic_source": "profiles/traffic.json (rocprofv3 FETCH_SIZE + WRITE_SIZE, raw KiB x 1024, per launch)",
            "kernel": kernel_name(args.codec),
            "kernel_ms": round(k_ms, 3),
            "algorithmic_bytes_per_launch": int(algo_bytes),
        },
        "roofline_decompress": {
            "bound": "hbm",
            "achieved": round(dec_achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(dec_achieved / HBM_PEAK_GBS, 5),
            "traffic": traffic_for("lzh_decompress_v2_kernel") if default_workload else None,
            "kernel": "lzh_decompress_v2_kernel",
            "kernel_ms": round(d_ms, 3),
        },
        "cpu_baseline": cpu,
        "ratio_pct": round(100 * ratio, 3),
        "comp_MBps": round(n / ((k_ms + f_ms) * 1e-3) / 1e6, 2),
        "decomp_MBps": round(n / (d_ms * 1e-3) / 1e6, 2),
        "stage_ms": {"compress_kernel": round(k_ms, 3), "scan_pack": round(f_ms, 3), "decompress": round(d_ms, 3)},
        "roundtrip_ok": roundtrip_ok,
    }
    res.update(result_extra)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
