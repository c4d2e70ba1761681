"""lzbench_amd/shard.py -- chunk sharding across ranks, one process per GPU.

Chunks are independent (reference _lzbench/lzbench.cpp:366-373: each chunk is compressed on its
own), so rank r of W takes the contiguous chunk range [r*K/W, (r+1)*K/W) of the lzbench chunk
list and compresses it on its own GPU.  The one exchange is SURVEY 8(e)'s single host-side
gather: the ranks all-gather their packed totals and chunk counts (a few bytes, control plane),
then every rank copies its packed slab and its compr_sizes straight into one shared host buffer
(a /dev/shm mapping) at its chunk-order offset -- the layout of lzbench's compbuf
(lzbench.cpp:266-298: chunk i at sum(clen[<i])).  No collective moves codec bytes -- unless the
ranks span hosts or /dev/shm lacks the room, where point-to-point sends to rank 0 take over.  The result is
byte-identical to the single-process chunk loop.  bench.py times the same gather on HBM-resident
slabs.
"""
from __future__ import annotations

import mmap
import os
import time
import uuid
from typing import Callable, Optional, Tuple

import numpy as np

def shard_range(nchunks: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous chunk range [c0, c1) owned by `rank`."""
    return nchunks * rank // world, nchunks * (rank + 1) // world


def shard_bytes(n: int, chunk_size: int, rank: int, world: int) -> Tuple[int, int]:
    """Byte range of the input owned by `rank` (chunk aligned)."""
    k = max((n + chunk_size - 1) // chunk_size, 1)
    c0, c1 = shard_range(k, rank, world)
    return min(c0 * chunk_size, n), min(c1 * chunk_size, n)


def _shm_usable(nbytes: int, world: int, group) -> Tuple[bool, str]:
    """The shared-buffer gather needs every rank on one host and room for the buffer in /dev/shm
    (tmpfs: a mapping past its free space raises SIGBUS on write).  Decided on rank 0 from every
    rank's hostname and its own statvfs, and broadcast so all ranks take the same path."""
    import socket
    import torch.distributed as dist
    hosts = [None] * world
    dist.all_gather_object(hosts, socket.gethostname(), group=group)
    verdict = [None]
    if (dist.get_rank(group) if group is not None else dist.get_rank()) == 0:
        why = ""
        if len(set(hosts)) > 1:
            why = "ranks on %d hosts" % len(set(hosts))
        else:
            try:
                st = os.statvfs("/dev/shm")
                free = st.f_bavail * st.f_frsize
                if free < nbytes + (64 << 20):
                    why = "/dev/shm has %d MiB free for %d MiB" % (free >> 20, nbytes >> 20)
            except OSError as e:
                why = "no /dev/shm (%s)" % e
        if os.environ.get("LZH_GATHER") == "collective":
            why = why or "LZH_GATHER=collective"
        verdict[0] = why
    src = 0 if group is None else dist.get_global_rank(group, 0)
    dist.broadcast_object_list(verdict, src=src, group=group)
    return verdict[0] == "", verdict[0]


def _gather_collective(p, c, sizes, counts, rank, world, group, keep):
    """Fallback: rank 0 receives the slabs one by one (point-to-point; CUDA tensors under nccl, host
    tensors under gloo) and writes each straight into one preallocated host buffer at its chunk-order
    offset: the device holds at most one received slab at a time, never world x the largest."""
    import torch
    import torch.distributed as dist
    nccl = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if nccl else torch.device("cpu")
    glob = (lambda r: r) if group is None else (lambda r: dist.get_global_rank(group, r))
    if p.is_cuda or nccl:
        torch.cuda.synchronize()
    dist.barrier(group=group)
    t = time.perf_counter()
    res = None
    if rank == 0:
        hp = torch.empty(sum(sizes), dtype=torch.uint8)
        hc = torch.empty(sum(counts), dtype=torch.int64)
        hp[:sizes[0]].copy_(p)
        hc[:counts[0]].copy_(c)
        rb = torch.empty(max(sizes[1:] + [1]), dtype=torch.uint8, device=dev) if nccl else None
        rc = torch.empty(max(counts[1:] + [1]), dtype=torch.int64, device=dev) if nccl else None
        pb, cb = sizes[0], counts[0]
        for r in range(1, world):
            if sizes[r]:
                if nccl:
                    dist.recv(rb[:sizes[r]], src=glob(r), group=group)
                    hp[pb:pb + sizes[r]].copy_(rb[:sizes[r]])
                else:
                    dist.recv(hp[pb:pb + sizes[r]], src=glob(r), group=group)
            if counts[r]:
                if nccl:
                    dist.recv(rc[:counts[r]], src=glob(r), group=group)
                    hc[cb:cb + counts[r]].copy_(rc[:counts[r]])
                else:
                    dist.recv(hc[cb:cb + counts[r]], src=glob(r), group=group)
            pb += sizes[r]
            cb += counts[r]
        if keep:
            res = (hp.numpy(), hc.numpy().astype(np.uint64))
    else:
        if sizes[rank]:
            dist.send(p.to(dev).contiguous(), dst=glob(0), group=group)
        if counts[rank]:
            dist.send(c.to(dev).contiguous(), dst=glob(0), group=group)
    el = torch.tensor([time.perf_counter() - t], dtype=torch.float64, device=dev)
    dist.all_reduce(el, op=dist.ReduceOp.MAX, group=group)
    return float(el.item()), res


def gather_slabs(packed, csizes, rank: int, world: int, group=None, keep: bool = True):
    """Place every rank's packed slab and compr_sizes in one shared host buffer in chunk order.

    packed: this rank's packed bytes (numpy u8 array, or a torch u8 tensor on the host or the GPU);
    csizes: its per-chunk compressed sizes (numpy / torch, any integer type).  Returns
    ({"ms", "bytes", "GBps", "path"} of the slab copies, max over ranks; (packed_all, csizes_all) on
    rank 0 when keep, else None).  "path" is "shm" (every rank copies its slab into one /dev/shm
    mapping) or "collective" (slabs sent to rank 0 one by one: ranks on several hosts, too little
    /dev/shm, or LZH_GATHER=collective)."""
    import torch
    import torch.distributed as dist

    def as_tensor(a, dtype):
        t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))
        return t.reshape(-1).to(dtype) if t.dtype != dtype else t.reshape(-1)

    p = as_tensor(packed, torch.uint8)
    c = as_tensor(csizes, torch.int64)
    meta = torch.tensor([p.numel(), c.numel()], dtype=torch.int64)
    if dist.get_backend(group) == "nccl":
        meta = meta.cuda()
    metas = [torch.zeros_like(meta) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    sizes = [int(m[0]) for m in metas]
    counts = [int(m[1]) for m in metas]
    grand, kall = sum(sizes), sum(counts)
    base, cbase = sum(sizes[:rank]), sum(counts[:rank])
    nbytes = grand + 8 * kall
    ok, why = _shm_usable(nbytes, world, group)
    if not ok:
        sec, res = _gather_collective(p, c, sizes, counts, rank, world, group, keep)
        ms = sec * 1e3
        return {"ms": round(ms, 3), "bytes": grand, "GBps": round(grand / max(sec, 1e-12) / 1e9, 2),
                "path": "collective", "why": why}, res
    # rank 0 names the buffer (unique per call, whatever the rendezvous) and tells the others
    name = [None]
    if rank == 0:
        name[0] = "/dev/shm/lzh_gather_%d_%s" % (os.getpid(), uuid.uuid4().hex)
    dist.broadcast_object_list(name, src=0 if group is None else dist.get_global_rank(group, 0), group=group)
    path = name[0]
    res = None
    fd = -1
    mm = None
    try:
        if rank == 0:
            with open(path, "wb") as f:
                f.truncate(max(nbytes, 1))
        dist.barrier(group=group)
        fd = os.open(path, os.O_RDWR)
        mm = mmap.mmap(fd, max(nbytes, 1))
        host = torch.frombuffer(mm, dtype=torch.uint8, count=max(nbytes, 1))
        if p.is_cuda:
            torch.cuda.synchronize()
        dist.barrier(group=group)
        t = time.perf_counter()
        if p.numel():
            host[base:base + p.numel()].copy_(p)
        if c.numel():
            host[grand + 8 * cbase:grand + 8 * (cbase + c.numel())].copy_(c.cpu().view(torch.uint8))
        if p.is_cuda:
            torch.cuda.synchronize()
        dist.barrier(group=group)
        el = torch.tensor([time.perf_counter() - t], dtype=torch.float64)
        if dist.get_backend(group) == "nccl":
            el = el.cuda()
        dist.all_reduce(el, op=dist.ReduceOp.MAX, group=group)
        if rank == 0 and keep:
            buf = np.frombuffer(mm, np.uint8, count=nbytes) if nbytes else np.zeros(0, np.uint8)
            res = (buf[:grand].copy(), buf[grand:].copy().view("<i8").astype(np.uint64))
            del buf
        del host
        dist.barrier(group=group)
    finally:
        if mm is not None:
            mm.close()
        if fd >= 0:
            os.close(fd)
        if rank == 0 and os.path.exists(path):
            os.unlink(path)
    ms = float(el.item()) * 1e3
    return {"ms": round(ms, 3), "bytes": grand, "GBps": round(grand / max(ms * 1e-3, 1e-9) / 1e9, 2), "path": "shm"}, res


def sharded_compress(data: np.ndarray, chunk_size: int, rank: int, world: int,
                     compress: Callable[[np.ndarray], Tuple[np.ndarray, np.ndarray]],
                     group=None) -> Optional[Tuple[np.ndarray, np.ndarray]]:
    """Compress this rank's shard with `compress(shard) -> (packed, csizes)` and gather every
    rank's slab into the shared host buffer.  Returns (packed, csizes) on rank 0, None elsewhere."""
    b0, b1 = shard_bytes(len(data), chunk_size, rank, world)
    packed, cs = compress(np.ascontiguousarray(data[b0:b1])) if b1 > b0 else (
        np.zeros(0, np.uint8), np.zeros(0, np.uint64))
    _, res = gather_slabs(packed, cs, rank, world, group=group)
    return res
