#!/usr/bin/env python3
"""bench.py -- the lzbench hot path on MI355X: lz4 -b64 over 1 GiB of synthetic text per GPU.

One step = one lzbench pass over the whole input (reference _lzbench/lzbench.cpp:384-393 and
:418-427): compress every 64 KiB chunk (HIP codec kernel, then size scan + packing with the
raw-store rule), then decompress every chunk from the packed stream.  Inputs are resident in
HBM when the timed region starts.  value = comp+decomp MB/s (MB = 1e6 B, lzbench.cpp:104-106)
= bytes processed by all ranks / (max over ranks of the timed wall time).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): one process per
GPU; rank r owns share r -- bytes [r x 1 GiB, (r+1) x 1 GiB) -- of ONE N GiB seed-12345 corpus, i.e.
its contiguous range of that corpus's lzbench chunk list (lzbench.cpp:366-373; weak scaling: 1 GiB
per GPU).  Every share, and the gathered whole, is checked against the reference chunk loop's digest
of exactly those bytes (tests/golden/fullsize.json, make_fullsize.py SHARED).  The only
exchange is the host-side gather of SURVEY.md 8(e): after the timed region the ranks all-gather
their packed totals (a few bytes, control plane), and each copies its packed slab straight into
one shared host buffer at its chunk-order offset (lzbench_amd/shard.py gather_slabs); that gather
is timed and reported (`gather`).  No collective touches the data path.  Rank 0 then also times
the in-process N-device product path (`e2e`: lzbench_hip_compress_batch / _decompress_batch with
ngpus = N over the N shards' bytes, what `lzbench_hip -gN` runs).

Also reported (rank 0):
  roofline / roofline_decompress  the codec kernels, HIP events on the stream they run on
  bit_exact                       the whole packed stream + compr_sizes vs the reference digest
                                  (tests/golden/fullsize.json) when the workload has one
  cpu_baseline                    the reference codec (oracle/_ref, built from the reference
                                  sources) on this host, 1 thread, lzbench semantics (N=1 only)
  cpu_baseline_all_cores          the same on every host core this process may use
  e2e                             host-to-host through the batched lzbench rows
                                  (lzbench_hip_compress_batch / _decompress_batch, ngpus = N) on
                                  the whole N-share corpus, beside the hipMemcpy
                                  round-trip bound (PCIe; never value)
  roofline_compress_stage         the whole compress stage (parse + emit + scan + pack) against
                                  the same N + C algorithmic bytes
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
BASELINE_METRIC = "comp+decomp MB/s, lz4 -b64 on 1 GiB; ratio + bit-exact vs CPU ref"
COMPRESS_KERNEL = {"lz4": "lzh_lz4_parse_kernel", "lz4fast": "lzh_lz4_parse_kernel",
                   "snappy": "lzh_snappy_parse_kernel",
                   "zstd": "lzh_zstd_match_kernel+lzh_zstd_entropy_kernel"}
# (zstd decodes in five kernels, and frames the split layout does not fit in a sixth: the stage)
# (the per-lane literal kernel comes in two widths, lzh_zstd_huf_kernel / lzh_zstd_huf8_kernel, picked by frame
# count; streams of 4096+ symbols go to lzh_zstd_hufpar_kernel; the sequence kernel runs beside them)
DECOMPRESS_KERNEL = {"zstd": "lzh_zstd_hdr_kernel+lzh_zstd_huf_kernel+lzh_zstd_huf8_kernel+lzh_zstd_hufpar_kernel"
                             "+lzh_zstd_seq_kernel+lzh_zstd_exec_kernel+lzh_zstd_decompress_kernel"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def size_label(n):
    return f"{n >> 30} GiB" if n % (1 << 30) == 0 else f"{n >> 20} MiB"


def metric_for(codec, chunk_kib, n, corpus, level):
    """BASELINE.json's metric string for the north-star workload; the same wording naming the
    codec, chunk size and corpus for every other workload."""
    if codec == "lz4" and chunk_kib == 64 and n == 1 << 30 and corpus == "text":
        return BASELINE_METRIC
    name = codec if codec not in ("lz4fast", "zstd") else f"{codec},{level}"
    return f"comp+decomp MB/s, {name} -b{chunk_kib} on {size_label(n)} {corpus}; ratio + bit-exact vs CPU ref"


def host_cpus():
    """(threads usable by this process, description): the affinity mask capped by the cgroup CPU
    quota (a GPU box exposes the whole machine in os.cpu_count() but grants a share of it)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    return usable, {"model": model, "nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota,
                    "threads_used_all_cores": usable}


def cpu_baseline(sample: np.ndarray, codec: str, chunk: int, level: int, iters: int, threads: int):
    """lzbench semantics on the host: best-of-iters compress pass + best-of-iters decompress
    pass over the sample (lzbench.cpp:379-469, -p1 fastest). Uses the reference build when
    present (kind 'reference'), else the repo's C restatement (kind 'port')."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    use_ref = O.have_ref() or codec == "zstd"
    n = len(sample)
    best_c = best_d = float("inf")
    packed = cs = None
    for _ in range(iters):
        t = time.perf_counter()
        packed, cs = O.compress_chunks(sample, codec, chunk, level, use_ref=use_ref, threads=threads)
        best_c = min(best_c, time.perf_counter() - t)
    r, out = None, None
    for _ in range(iters):
        t = time.perf_counter()
        r, out = O.decompress_chunks(packed, cs, n, codec, chunk, use_ref=use_ref, threads=threads)
        best_d = min(best_d, time.perf_counter() - t)
    ok = r == n and bool((out == sample).all())
    lib = {"lz4": "lz4 1.9.3", "lz4fast": "lz4 1.9.3", "snappy": "snappy 1.1.8", "zstd": "zstd 1.5.2"}[codec]
    return {
        "value": round(n / (best_c + best_d) / 1e6, 2),
        "unit": "MB/s",
        "cores": max(threads, 1),
        "kind": "reference" if use_ref else "port",
        "sample": f"{size_label(n)} = the whole per-GPU input, -b{chunk >> 10}, best of {iters} compress + {iters} "
                  f"decompress passes ({lib + ' compiled from the reference sources' if use_ref else 'oracle C restatement'}"
                  f", {max(threads, 1)} thread{'s' if threads > 1 else ''})",
        "comp_MBps": round(n / best_c / 1e6, 2),
        "decomp_MBps": round(n / best_d / 1e6, 2),
        "roundtrip_ok": ok,
    }


_HASHES = None


def _loaded_hashes():
    """kernel code hashes of the library this process loads (lzbench_amd.kernel_hash)"""
    global _HASHES
    if _HASHES is None:
        import lzbench_amd
        from lzbench_amd import kernel_hash
        try:
            _HASHES = kernel_hash.kernel_hashes(lzbench_amd.LIB_PATH)
        except (OSError, ValueError):
            _HASHES = {}
    return _HASHES


def traffic_for(kernel, workload):
    """(HBM-side bytes per dispatch of `kernel`, None) from the committed PMC profiles (profiles/traffic*.json,
    written by tools/pmc_traffic.sh: FETCH_SIZE and WRITE_SIZE in separate rocprofv3 passes on the
    same workload; one file per workload), or (None, reason) when no profile covers this kernel/workload or the
    profile was taken of other machine code than the loaded library's (each profile records the code hash of
    every kernel it measured, lzbench_amd/kernel_hash.py)."""
    import glob
    have = _loaded_hashes()
    reason = f"no profiles/traffic*.json for {kernel} on {workload}"
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic*.json"))):
        try:
            with open(path) as f:
                t = json.load(f)
            if t.get("workload_key") != workload:
                continue
            # a stage of several kernels ("a+b"): the sum over the kernels the profile holds (a kernel
            # no dispatch of which ran in the profiled pass has no entry and contributes nothing)
            parts = {k: t["kernels"].get(k) for k in kernel.split("+")}
            if all(p is None for p in parts.values()):
                continue
            stale = [k for k, p in parts.items()
                     if p is not None and (p.get("kernel_hash") is None or p["kernel_hash"] != have.get(k))]
            if stale:
                reason = (f"{os.path.relpath(path, ROOT)} measured other code of {', '.join(stale)} "
                          f"(profile hash {parts[stale[0]].get('kernel_hash')}, loaded {have.get(stale[0])})")
                continue
            return int(sum(p["traffic_bytes_per_dispatch"] for p in parts.values() if p is not None)), None
        except (OSError, KeyError, ValueError):
            continue
    return None, reason


def fullsize_digest(corpus, codec, chunk, level, n, seed, offset=0):
    """the reference chunk loop's digest of corpus bytes [offset, offset + n) (tests/golden/fullsize.json)"""
    path = os.path.join(ROOT, "tests", "golden", "fullsize.json")
    try:
        for e in json.load(open(path)):
            lvl = level if codec in ("lz4fast", "zstd") else (1 if codec == "lz4" else 0)
            if (e["corpus"], e["codec"], e["chunk"], e["level"], e["size"], e["seed"], e.get("offset", 0)) == \
                    (corpus, codec, chunk, lvl, n, seed, offset):
                return e
    except (OSError, ValueError):
        pass
    return None


def sha(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def e2e_rows(L, host, codec, chunk, level, ngpus, iters, dig=None):
    """Host-to-host through the batched lzbench rows (what lzbench_hip -b -g<ngpus> runs): best of
    `iters` compress_batch and decompress_batch passes over `host` (its chunk list sharded over
    ngpus devices, api.cpp make_plan), and the hipMemcpy round trip (H2D + D2H of the same bytes,
    pinned, one device) as the PCIe bound beside them.  dig: the reference digest of `host` itself:
    the whole packed output and compr_sizes must hash to it."""
    import torch
    n = len(host)
    cs = L.chunk_sizes_for(n, chunk)
    out = np.empty(L.get_compress_bound(n) + 64, np.uint8)
    comp = np.zeros(len(cs), np.uint64)
    back = np.empty(n + L.PAD_SIZE, np.uint8)
    lvl = level if codec in ("lz4fast", "zstd") else (1 if codec == "lz4" else 0)
    lib = L.lib()
    best_c = best_d = float("inf")
    tot = 0
    with L._Row(codec, chunk, lvl, ngpus) as row:
        for _ in range(iters):
            t = time.perf_counter()
            tot = lib.lzbench_hip_compress_batch(host.ctypes.data, cs.ctypes.data, len(cs), out.ctypes.data, len(out),
                                                 comp.ctypes.data, lvl, ngpus, row.wm)
            best_c = min(best_c, time.perf_counter() - t)
        for _ in range(iters):
            t = time.perf_counter()
            r = lib.lzbench_hip_decompress_batch(out.ctypes.data, comp.ctypes.data, cs.ctypes.data, len(cs),
                                                 back.ctypes.data, len(back), lvl, ngpus, row.wm)
            best_d = min(best_d, time.perf_counter() - t)
    ok = tot > 0 and r == n and bool((back[:n] == host).all())
    exact = None
    if dig is not None and tot > 0 and dig["size"] == n:
        exact = tot == dig["packed_bytes"] and sha(comp.astype("<u8")) == dig["csizes_sha256"] and \
            sha(out[:tot]) == dig["packed_sha256"]
    del back
    pin = torch.from_numpy(host[:min(n, 1 << 30)]).pin_memory()
    n1 = len(pin)
    dev = torch.empty(n1, dtype=torch.uint8, device="cuda")
    hb = torch.empty(n1, dtype=torch.uint8).pin_memory()
    best_m = float("inf")
    for _ in range(iters):
        torch.cuda.synchronize()
        t = time.perf_counter()
        dev.copy_(pin, non_blocking=True)
        hb.copy_(dev, non_blocking=True)
        torch.cuda.synchronize()
        best_m = min(best_m, time.perf_counter() - t)
    del pin, dev, hb
    return {
        "comp_MBps": round(n / best_c / 1e6, 2),
        "decomp_MBps": round(n / best_d / 1e6, 2),
        "comp+decomp_MBps": round(n / (best_c + best_d) / 1e6, 2),
        "hipMemcpy_roundtrip_MBps": round(n1 / best_m / 1e6, 2),
        "hipMemcpy_roundtrip_note": "one device, pinned, %d bytes" % n1,
        "ngpus": ngpus,
        "roundtrip_ok": ok,
        "bit_exact": exact,
        "bytes": n,
        "note": "host pageable buffers (page-locked once per row), H2D + kernels + D2H pipelined over "
                "128 MiB sub-batches; best of %d passes; PCIe-bound, reported beside value, never as value" % iters,
    }


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--codec", default="lz4", choices=["lz4", "lz4fast", "snappy", "zstd"])
    ap.add_argument("--level", type=int, default=1, help="lz4fast acceleration / zstd level")
    ap.add_argument("--chunk-kib", type=int, default=64)
    ap.add_argument("--size-mib", type=int, default=1024, help="input bytes per GPU")
    ap.add_argument("--corpus", default="text", choices=["text", "json", "mixed", "random", "binary"])
    ap.add_argument("--cpu-iters", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
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
        # (gloo prints "[Gloo] Rank r is connected to ..." on the process's stdout while it connects:
        # send it to stderr, so that rank 0's stdout is the one JSON line)
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend=args.backend)
        finally:
            os.dup2(saved, 1)
            os.close(saved)

    import lzbench_amd as L

    n = args.size_mib << 20
    chunk = args.chunk_kib << 10
    seed = 12345                       # the digest-pinned corpus (see docstring)
    if world > 1 and (n % (16 << 20) or n % chunk):
        raise SystemExit("bench.py: at N > 1 the per-GPU size must be a multiple of 16 MiB and of the chunk size "
                         "(rank r owns bytes [r n, (r+1) n) of one corpus)")
    t = time.perf_counter()
    host = L.datagen(args.corpus, n, seed=seed, offset=rank * n)   # share `rank` of one world x n corpus
    log(f"[rank {rank}] generated share {rank} ({n >> 20} MiB) of {world * n >> 20} MiB {args.corpus} "
        f"in {time.perf_counter() - t:.1f}s")
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
    d_in[:n].copy_(torch.from_numpy(host))
    codec = L.DeviceCodec(args.codec, n, chunk, level=args.level)
    stream = torch.cuda.current_stream()

    nsteps = args.warmup + args.steps
    ev = [[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in range(nsteps)]

    def step(i):
        e = ev[i]
        e[0].record(stream)
        codec.compress_stage(d_in, 1)            # parse kernel: the dominant kernel (roofline)
        e[1].record(stream)
        codec.compress_stage(d_in, 2)            # block emission (LZ4 / snappy) from the parse records
        e[4].record(stream)
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
    x_ms = float(np.mean([e[1].elapsed_time(e[4]) for e in timed]))
    f_ms = float(np.mean([e[4].elapsed_time(e[2]) for e in timed]))
    d_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in timed]))
    comp_total = codec.packed_total()
    k_chunks = int(codec.k)
    roundtrip_ok = bool(torch.equal(codec.out[:n], d_in[:n])) and bool((codec.status >= 0).all().item())
    ratio = comp_total / n

    result_extra = {}
    whole = fullsize_digest(args.corpus, args.codec, chunk, args.level, world * n, seed) if world > 1 else None
    if dist:
        from lzbench_amd.shard import gather_slabs
        g, res = gather_slabs(codec.packed[:comp_total], codec.csizes[:codec.k], rank, world, keep=whole is not None)
        g["how"] = ("all_gather of packed totals, then each rank copies its HBM slab (and its compr_sizes) into one "
                    "shared host buffer at its chunk-order offset (lzbench_amd/shard.py gather_slabs); timed after "
                    "the timed region, max over ranks")
        if rank == 0 and res is not None:
            # the gathered whole (every share in chunk order) against the digest of the whole corpus
            g["bit_exact_whole"] = bool(len(res[0]) == whole["packed_bytes"] and sha(res[0]) == whole["packed_sha256"]
                                        and sha(res[1].astype("<u8")) == whole["csizes_sha256"])
            g["whole_bytes"] = world * n
        del res
        result_extra["gather"] = g

    # bit-exactness of the WHOLE output vs the reference chunk loop's digest of this rank's share
    dig = fullsize_digest(args.corpus, args.codec, chunk, args.level, n, seed, offset=rank * n)
    exact = None
    if dig is not None:
        cs64 = codec.csizes.cpu().numpy().astype("<u8")
        exact = bool(comp_total == dig["packed_bytes"] and sha(cs64) == dig["csizes_sha256"]
                     and sha(codec.packed[:comp_total].cpu().numpy()) == dig["packed_sha256"])
    ranks_exact = [exact]
    if dist:
        flag = torch.tensor([-1 if exact is None else int(exact)], dtype=torch.int64)
        flags = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(flags, flag)
        ranks_exact = [None if int(f.item()) < 0 else bool(f.item()) for f in flags]
    if all(x is not None for x in ranks_exact):
        result_extra["bit_exact"] = all(ranks_exact)
        result_extra["bit_exact_ranks"] = ranks_exact
        result_extra["bit_exact_bytes"] = n * world
        result_extra["bit_exact_against"] = ("tests/golden/fullsize.json (reference chunk loop, oracle/_ref): "
                                             "each rank's share, offset r x size")
    else:
        result_extra["bit_exact"] = None
        result_extra["bit_exact_ranks"] = ranks_exact
        result_extra["bit_exact_against"] = "no committed reference digest for this workload (or for some share)"

    cpu = None
    usable, cpuinfo = host_cpus()
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(host, args.codec, chunk, args.level, args.cpu_iters, 0)
        result_extra["cpu_baseline_all_cores"] = cpu_baseline(host, args.codec, chunk, args.level, args.cpu_iters,
                                                              usable)
    result_extra["host_cpu"] = cpuinfo
    if not args.no_e2e:
        # the in-process product path over all N devices, by rank 0 while the other ranks wait
        # (host memory on rank 0: the N-copy input plus its packed output and the decode buffer, about
        # 3N GiB at the default 1 GiB per GPU -- 24 GiB at N = 8, well inside a node's RAM)
        del d_in, codec
        torch.cuda.empty_cache()
        if dist:
            dist.barrier()
        if rank == 0:
            big = host if world == 1 else L.datagen(args.corpus, world * n, seed=seed)
            result_extra["e2e"] = e2e_rows(L, big, args.codec, chunk, args.level, world, 3, dig if world == 1 else whole)
            del big
        if dist:
            dist.barrier()

    algo_bytes = n + comp_total                      # compress reads N, writes C
    achieved = algo_bytes / (k_ms * 1e-3) / 1e9
    dec_achieved = algo_bytes / (d_ms * 1e-3) / 1e9   # decompress reads C, writes N
    wkey = f"{args.codec}/{args.level}/{args.chunk_kib}/{args.corpus}/{n}"
    total_bytes = world * n * args.steps
    value = total_bytes / elapsed / 1e6
    kname = COMPRESS_KERNEL[args.codec]
    dname = DECOMPRESS_KERNEL.get(args.codec)
    if dname is None:   # LZ4 / snappy: the output-window variant the launcher picks for this many chunks
        import ctypes
        win = {8192: "lzh_decompress_w8k_kernel", 16384: "lzh_decompress_w16k_kernel"}

        def wkernel(nchunks):
            return win.get(L.lib().lzh_debug_decode_window(ctypes.c_uint32(nchunks)), "lzh_decompress_v2_kernel")
        k_all = -(-n // chunk)
        frags = -(-chunk // 65536)
        if args.codec == "snappy" and 8 <= frags <= 64:   # split scan, fragments, join, the chunks decoded whole
            names = ["lzh_snappy_split_kernel", wkernel(k_all * frags), "lzh_snappy_join_kernel", wkernel(k_all)]
            dname = "+".join(dict.fromkeys(names))
        else:
            dname = wkernel(k_all)
    tr_c, why_c = traffic_for(kname, wkey)
    tr_d, why_d = traffic_for(dname, wkey)
    res = {
        "metric": metric_for(args.codec, args.chunk_kib, n, args.corpus, args.level),
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
        "data": f"synthetic {args.corpus} corpus (SURVEY.md 8(d) stand-in; enwik8/Silesia unavailable offline): "
                f"rank r owns share r ({size_label(n)}) of one {size_label(world * n)} seed-12345 corpus, resident in HBM",
        "config": {
            "workload": f"{args.codec}{',' + str(args.level) if args.codec in ('lz4fast', 'zstd') else ''} "
                        f"-b{args.chunk_kib} on {size_label(n)} {args.corpus} per GPU, comp+decomp pass",
            "codec": args.codec,
            "chunk_kib": args.chunk_kib,
            "bytes_per_gpu": n,
            "chunks_per_gpu": k_chunks,
            "parallelism": f"chunk-sharded x{world} (contiguous shard per GPU, host-side gather, no collective)",
        },
        "roofline": {
            "bound": "hbm",
            "achieved": round(achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": tr_c,
            "traffic_source": "profiles/traffic*.json (rocprofv3 FETCH_SIZE + WRITE_SIZE, separate passes, per launch; "
                              "only for the machine code the profile measured)",
            **({"traffic_null_reason": why_c} if tr_c is None else {}),
            "kernel": kname,
            "kernel_ms": round(k_ms, 3),
            "algorithmic_bytes_per_launch": int(algo_bytes),
        },
        "roofline_compress_stage": {
            "bound": "hbm",
            "achieved": round(algo_bytes / ((k_ms + x_ms + f_ms) * 1e-3) / 1e9, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(algo_bytes / ((k_ms + x_ms + f_ms) * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
            "kernels": f"{kname} + emit + lzh_scan_kernel + lzh_pack_kernel",
            "stage_ms": round(k_ms + x_ms + f_ms, 3),
        },
        "roofline_decompress": {
            "bound": "hbm",
            "achieved": round(dec_achieved, 2),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(dec_achieved / HBM_PEAK_GBS, 5),
            "traffic": tr_d,
            **({"traffic_null_reason": why_d} if tr_d is None else {}),
            "kernel": dname,
            "kernel_ms": round(d_ms, 3),
        },
        "cpu_baseline": cpu,
        "ratio_pct": round(100 * ratio, 3),
        "comp_MBps": round(n / ((k_ms + x_ms + f_ms) * 1e-3) / 1e6, 2),
        "decomp_MBps": round(n / (d_ms * 1e-3) / 1e6, 2),
        "stage_ms": {"compress_kernel": round(k_ms, 3), "emit_kernel": round(x_ms, 3), "scan_pack": round(f_ms, 3),
                     "decompress": round(d_ms, 3)},
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
