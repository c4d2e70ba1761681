"""lzbench_amd/shard.py -- chunk sharding across ranks, one process per GPU.

Chunks are independent (reference _lzbench/lzbench.cpp:366-373: each chunk is compressed on its
own), so rank r of W takes the contiguous chunk range [r*K/W, (r+1)*K/W) of the lzbench chunk
list, compresses it on its own GPU, and the packed slabs are gathered to rank 0 in chunk order
(the host-side gather; no collective on the data path beyond moving the finished bytes).  The
result is byte-identical to the single-process chunk loop.
"""
from __future__ import annotations

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


def sharded_compress(data: np.ndarray, chunk_size: int, rank: int, world: int,
                     compress: Callable[[np.ndarray], Tuple[np.ndarray, np.ndarray]],
                     group=None) -> Optional[Tuple[np.ndarray, np.ndarray]]:
    """Compress this rank's shard with `compress(shard) -> (packed, csizes)` and gather every
    rank's slab to rank 0.  Returns (packed, csizes) on rank 0, None elsewhere."""
    import torch
    import torch.distributed as dist

    b0, b1 = shard_bytes(len(data), chunk_size, rank, world)
    packed, cs = compress(np.ascontiguousarray(data[b0:b1])) if b1 > b0 else (
        np.zeros(0, np.uint8), np.zeros(0, np.uint64))
    # sizes first (a few KB), then the slabs themselves: rank 0 lays them out by prefix sums
    meta = torch.tensor([len(packed), len(cs)], dtype=torch.int64)
    metas = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(metas, meta, group=group)
    maxp = int(max(m[0] for m in metas)) or 1
    maxc = int(max(m[1] for m in metas)) or 1
    pbuf = torch.zeros(maxp, dtype=torch.uint8)
    pbuf[: len(packed)] = torch.from_numpy(packed)
    cbuf = torch.zeros(maxc, dtype=torch.int64)
    cbuf[: len(cs)] = torch.from_numpy(cs.astype(np.int64))
    plist = [torch.zeros(maxp, dtype=torch.uint8) for _ in range(world)] if rank == 0 else None
    clist = [torch.zeros(maxc, dtype=torch.int64) for _ in range(world)] if rank == 0 else None
    dist.gather(pbuf, plist, dst=0, group=group)
    dist.gather(cbuf, clist, dst=0, group=group)
    if rank != 0:
        return None
    packed_all = np.concatenate([plist[r][: int(metas[r][0])].numpy() for r in range(world)])
    cs_all = np.concatenate([clist[r][: int(metas[r][1])].numpy() for r in range(world)]).astype(np.uint64)
    return packed_all, cs_all
