"""GPU: the batched lzbench rows' sharding and gather (api.cpp run_compress / run_decompress) with
G = 1, 2, 4, 8 logical shards on one device, buffer sizing edge cases (one chunk covering the
whole input = lzbench without -b, lzbench.cpp:816), the device-resident API's capacity checks,
and the multi-rank shard/gather protocol with the HIP codec on every rank.  Expected bytes come
from the oracle (tests/test_oracle.py pins it to the reference build).  Run with -m gpu."""
import os
import socket

import numpy as np
import pytest

import oracle_lib as O
import lzbench_amd as L

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    return torch


@pytest.mark.parametrize("ngpus", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("codec,chunk", [("lz4", 65536), ("snappy", 262144), ("lz4", 131072)])
def test_sharded_batch_rows_equal_single_loop(torch_cuda, codec, chunk, ngpus):
    """lzbench_compress semantics (lzbench.cpp:266-298): chunk i packed at sum(clen[<i]) no matter
    how the chunk list is split over shards; the decode scatters the same offsets back."""
    n = 40 * chunk + 4321                      # ragged tail; several sub-batches per shard at G=8
    data = L.datagen("mixed", n, seed=ngpus)
    ep, ec = O.compress_chunks(data, codec, chunk)
    packed, cs = L.compress_chunks(data, codec, chunk, ngpus=ngpus)
    assert (cs == ec).all()
    assert len(packed) == len(ep) and (packed == ep).all()
    out = L.decompress_chunks(packed, cs, n, codec, chunk, ngpus=ngpus)
    assert (out == data).all()


def test_sharded_large_sub_batches(torch_cuda):
    """More than one 128 MiB sub-batch per shard (pipelined copy/compute/copy) at G = 2."""
    n = (300 << 20) + 77
    data = L.datagen("text", n, seed=5)
    ep, ec = O.compress_chunks(data, "lz4", 65536, threads=8)
    packed, cs = L.compress_chunks(data, "lz4", 65536, ngpus=2)
    assert (cs == ec).all() and len(packed) == len(ep) and (packed == ep).all()
    out = L.decompress_chunks(packed, cs, n, "lz4", 65536, ngpus=2)
    assert (out == data).all()


def test_eight_shards_north_star_digest(torch_cuda):
    """The in-process -g8 product path (api.cpp make_plan: 128 MiB sub-batches dealt round-robin to
    8 logical shards, per-shard copy / kernel / copy streams, host gather in chunk order) on the whole
    1 GiB north-star input: packed stream and compr_sizes equal the reference chunk loop's digest
    (tests/golden/fullsize.json), and the 8-shard decode round-trips."""
    import hashlib
    import json
    big = [e for e in json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")))
           if (e["corpus"], e["codec"], e["chunk"], e["size"]) == ("text", "lz4", 65536, 1 << 30)][0]
    data = L.datagen("text", big["size"], seed=big["seed"])
    packed, cs = L.compress_chunks(data, "lz4", 65536, ngpus=8)
    assert len(packed) == big["packed_bytes"]
    assert hashlib.sha256(cs.astype("<u8").tobytes()).hexdigest() == big["csizes_sha256"]
    assert hashlib.sha256(packed.tobytes()).hexdigest() == big["packed_sha256"]
    out = L.decompress_chunks(packed, cs, len(data), "lz4", 65536, ngpus=8)
    assert (out == data).all()


def _whole_corpora():
    import json
    return [e for e in json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")))
            if e.get("shares") == 8]


@pytest.mark.parametrize("big", _whole_corpora(),
                         ids=lambda b: f"{b['corpus']}{b['size'] >> 30}g-{b['codec']}{b['level']}-b{b['chunk'] >> 10}")
def test_eight_shards_whole_corpus_digest(torch_cuda, big):
    """BASELINE.json's 8-GPU workloads as stated -- config 4: 8 GiB of JSON logs, lz4 and snappy -b64; config 5:
    4 GiB mixed, zstd-1 -b128; and the north star's 8 x 1 GiB text -- as ONE corpus, one lzbench chunk list
    (lzbench.cpp:366-373), through the -g8 product path on one device (8 logical shards, api.cpp make_plan):
    the whole packed stream and compr_sizes equal the reference chunk loop's digest of the whole corpus
    (make_fullsize.py SHARED), and the 8-shard decode round-trips."""
    import hashlib
    data = L.datagen(big["corpus"], big["size"], seed=big["seed"])
    packed, cs = L.compress_chunks(data, big["codec"], big["chunk"], big["level"], ngpus=8)
    assert len(packed) == big["packed_bytes"]
    assert hashlib.sha256(cs.astype("<u8").tobytes()).hexdigest() == big["csizes_sha256"]
    assert hashlib.sha256(packed.tobytes()).hexdigest() == big["packed_sha256"]
    out = L.decompress_chunks(packed, cs, len(data), big["codec"], big["chunk"], ngpus=8)
    assert (out == data).all()


@pytest.mark.parametrize("codec", ["lz4", "snappy"])
def test_single_chunk_whole_input_row(torch_cuda, codec):
    """lzbench without -b: one chunk = the whole file (chunk_size clamped to the file size).
    The per-chunk row is called with insize = the whole input; buffers must be sized from the
    bytes actually present, not from a sub-batch of 1 024 such chunks."""
    lib = L.lib()
    data = L.datagen("json", 3 << 20, seed=2)
    n = len(data)
    init = getattr(lib, f"lzbench_hip_{codec}_init")
    wm = init(1_790_000_000, 0, 1)     # lzbench.cpp:816 default chunk size, clamped later
    assert wm
    try:
        out = np.zeros(L.get_compress_bound(n), np.uint8)
        clen = getattr(lib, f"lzbench_hip_{codec}_compress")(data.ctypes.data, n, out.ctypes.data, len(out), 0, 0, wm)
        exp = O.lz4_compress(data) if codec == "lz4" else O.snappy_compress(data)
        assert clen == len(exp) and out[:clen].tobytes() == exp
        back = np.zeros(n + L.PAD_SIZE, np.uint8)
        dlen = getattr(lib, f"lzbench_hip_{codec}_decompress")(out.ctypes.data, clen, back.ctypes.data, n, 0, 0, wm)
        assert dlen == n and (back[:n] == data).all()
        # the batched row with a chunk larger than the input
        cs = np.array([n], np.uint64)
        comp = np.zeros(1, np.uint64)
        tot = lib.lzbench_hip_compress_batch(data.ctypes.data, cs.ctypes.data, 1, out.ctypes.data, len(out),
                                             comp.ctypes.data, 1 if codec == "lz4" else 0, 1, wm)
        assert tot == len(exp) and int(comp[0]) == len(exp)
    finally:
        lib.lzbench_hip_deinit(wm)


def test_short_decode_reported_as_error(torch_cuda):
    """A stream that decodes to fewer bytes than its chunk must not pass as a full chunk: the
    row returns an error instead of the requested size (lzbench.cpp:433-437 length check)."""
    lib = L.lib()
    data = L.datagen("text", 65536, seed=4)
    short = np.frombuffer(O.snappy_compress(data[:60000].copy()), np.uint8).copy()   # varint says 60000
    wm = lib.lzbench_hip_snappy_init(65536, 0, 1)
    try:
        back = np.zeros(65536 + 64, np.uint8)
        r = lib.lzbench_hip_snappy_decompress(short.ctypes.data, len(short), back.ctypes.data, 65536, 0, 0, wm)
        assert r != 65536 and r <= 0
    finally:
        lib.lzbench_hip_deinit(wm)


def test_device_api_rejects_short_packed_capacity(torch_cuda):
    torch = torch_cuda
    n = 1 << 20
    data = L.datagen("random", n, seed=1)
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
    d_in[:n].copy_(torch.from_numpy(data))
    dc = L.DeviceCodec("lz4", n, 65536)
    dc.packed = dc.packed[: n // 2]            # far below lzh_max_packed_bytes
    with pytest.raises(RuntimeError, match="-3"):
        dc.compress(d_in)


def test_rows_restore_current_device(torch_cuda):
    torch = torch_cuda
    dev = torch.cuda.device_count() - 1
    torch.cuda.set_device(dev)
    try:
        data = L.datagen("text", 1 << 20, seed=3)
        packed, cs = L.compress_chunks(data, "lz4", 65536, ngpus=2)
        assert torch.cuda.current_device() == dev
        ep, ec = O.compress_chunks(data, "lz4", 65536)
        assert (packed == ep).all()
    finally:
        torch.cuda.set_device(0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, codec, chunk, n, q):
    import torch
    import torch.distributed as dist
    import lzbench_amd as L2
    from lzbench_amd.shard import sharded_compress
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(rank % torch.cuda.device_count())
    dist.init_process_group("gloo", rank=rank, world_size=world)
    data = L2.datagen("json", n, seed=78)
    res = sharded_compress(data, chunk, rank, world, lambda shard: L2.compress_chunks(shard, codec, chunk))
    if rank == 0:
        q.put((res[0].tobytes(), res[1].tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("codec,chunk", [("lz4", 65536), ("snappy", 262144)])
def test_two_rank_hip_shard_gather_equals_single(torch_cuda, codec, chunk):
    """The torchrun layout (one process per GPU, shard.py) with the HIP codec on each rank."""
    import torch.multiprocessing as mp
    n = 9 * chunk + 999
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, codec, chunk, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    packed, cs = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    data = L.datagen("json", n, seed=78)
    ep, ec = O.compress_chunks(data, codec, chunk)
    assert np.frombuffer(packed, np.uint8).tobytes() == ep.tobytes()
    assert cs == ec.tolist()
