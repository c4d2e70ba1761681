"""CPU, world_size 2 over gloo: the chunk-sharded multi-rank path gathers to a
result byte-identical to the single-process lzbench chunk loop.  Each rank's codec here is the
CPU checker (no GPU in this container); on the GPU box the same protocol runs with the HIP codec
(tests/test_gpu_parity.py covers that codec bit for bit)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_lib as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, codec, chunk, n, q, hip=False, gather_mode=None):
    import torch.distributed as dist
    import lzbench_amd as L
    from lzbench_amd.shard import sharded_compress
    if gather_mode:
        os.environ["LZH_GATHER"] = gather_mode
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = L.datagen("json", n, seed=77)
    if hip:   # the HIP codec through the C-ABI on this rank's device (one GPU box: both ranks on cuda:0)
        import torch
        torch.cuda.set_device(rank % torch.cuda.device_count())
        fn = lambda shard: L.compress_chunks(shard, codec, chunk)
    else:
        fn = lambda shard: O.compress_chunks(shard, codec, chunk)
    res = sharded_compress(data, chunk, rank, world, fn)
    # max-over-ranks timing reduction of bench.py's control plane
    import torch
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        q.put((res[0].tobytes(), res[1].tolist(), float(t.item())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("codec,chunk,mode", [("lz4", 65536, None), ("snappy", 262144, None),
                                              ("lz4", 65536, "collective")])
def test_two_rank_shard_gather_equals_single(codec, chunk, mode):
    """mode None: the shared /dev/shm buffer; "collective": the dist.gather fallback that ranks on
    several hosts (or a /dev/shm too small for the buffer) take -- forced here by LZH_GATHER."""
    import lzbench_amd as L
    n = 3 * chunk + 12345                       # ragged tail, uneven split across ranks
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, codec, chunk, n, q, False, mode)) for r in range(2)]
    for p in procs:
        p.start()
    packed, cs, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = L.datagen("json", n, seed=77)
    ep, ec = O.compress_chunks(data, codec, chunk)
    assert np.frombuffer(packed, np.uint8).tobytes() == ep.tobytes()
    assert cs == ec.tolist()
    assert tmax == 2.0


@pytest.mark.parametrize("world,nchunks", [(4, 7), (8, 5)])
def test_more_ranks_shard_gather_equals_single(world, nchunks):
    """the N=4 / N=8 launches of bench.py --gpus N rehearsed on gloo: uneven shares, and at N=8 with 5 chunks
    (4 full + a ragged tail) three ranks own no chunk at all; rank 0's gather is still the single-process loop's
    output byte for byte, and the max-over-ranks reduction sees every rank"""
    import lzbench_amd as L
    chunk = 65536
    n = (nchunks - 1) * chunk + 777
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, "lz4", chunk, n, q, False, None)) for r in range(world)]
    for p in procs:
        p.start()
    packed, cs, tmax = q.get(timeout=180)
    for p in procs:
        p.join(timeout=90)
        assert p.exitcode == 0
    data = L.datagen("json", n, seed=77)
    ep, ec = O.compress_chunks(data, "lz4", chunk)
    assert np.frombuffer(packed, np.uint8).tobytes() == ep.tobytes()
    assert cs == ec.tolist()
    assert tmax == float(world)


@pytest.mark.gpu
@pytest.mark.parametrize("codec,chunk", [("lz4", 65536), ("snappy", 262144), ("lz4frame", 65536)])
def test_two_rank_shard_gather_hip_codec(codec, chunk):
    """The same protocol with the HIP codec on each rank (gloo control plane, host gather):
    byte-identical to the single-process CPU chunk loop."""
    import torch
    import lzbench_amd as L
    if torch.cuda.device_count() < 1:   # (device_count does not initialise the GPU in this parent)
        pytest.skip("no HIP device")
    n = 3 * chunk + 12345
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, codec, chunk, n, q, True)) for r in range(2)]
    for p in procs:
        p.start()
    packed, cs, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = L.datagen("json", n, seed=77)
    oc = {"lz4frame": "lz4f"}.get(codec, codec)
    ep, ec = O.compress_chunks(data, oc, chunk, 0 if codec == "lz4frame" else 1)
    assert np.frombuffer(packed, np.uint8).tobytes() == ep.tobytes()
    assert cs == ec.tolist()


def _gather_path_worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    from lzbench_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    host = socket.gethostname
    if rank == 1:   # rank 1 pretends to live on another host: the shared buffer is not an option
        socket.gethostname = lambda: "elsewhere"
    info, res = shard.gather_slabs(np.full(10 + rank, rank + 1, np.uint8), np.array([10 + rank]), rank, world)
    socket.gethostname = host
    if rank == 0:
        q.put((info["path"], info.get("why", ""), res[0].tolist(), res[1].tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_falls_back_across_hosts():
    """with ranks on two hosts the /dev/shm gather cannot work (the other host's ranks
    cannot open the file), so every rank takes the dist.gather path, chosen on rank 0 and broadcast."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_path_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    path, why, packed, cs = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert path == "collective" and "2 hosts" in why
    assert packed == [1] * 10 + [2] * 11 and cs == [10, 11]


def test_shard_ranges_cover_all_chunks():
    from lzbench_amd.shard import shard_range, shard_bytes
    for k in (1, 2, 7, 16384):
        for w in (1, 2, 3, 8):
            rs = [shard_range(k, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == k
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
    assert shard_bytes(200_000, 65536, 1, 2) == (131072, 200_000)
