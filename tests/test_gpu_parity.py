"""GPU parity: the HIP codecs (through the C-ABI) against the reference's golden vectors and the
oracle, bit for bit, plus size-independent properties at full size.  Run with -m gpu."""
import ctypes as C

import numpy as np
import pytest

import golden_data as G
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


def gpu_block(codec, data, acc=1):
    """One chunk covering the whole input through the batched row."""
    n = len(data)
    chunk = max(n, 1)
    name = "lz4fast" if (codec == "lz4" and acc > 1) else codec
    packed, cs = L.compress_chunks(data, name, chunk, level=acc)
    return packed, cs


@pytest.mark.parametrize("case", [c for c in G.block_cases() if c["n"] > 0], ids=lambda c: c["key"])
def test_block_vs_golden(torch_cuda, case):
    data = G.inp(case["input"])[: case["n"]].copy()
    packed, cs = gpu_block(case["codec"], data, case["acc"])
    if int(cs[0]) == case["n"] and case["csize"] != case["n"]:
        pytest.fail("stored raw although the reference output differs in size")
    if int(cs[0]) == case["n"]:
        # lzbench raw-store rule: clen == part -> the chunk is the input bytes
        assert case["csize"] == case["n"] and (packed == data).all()
    else:
        assert G.check_block(case, packed.tobytes())
    out = L.decompress_chunks(packed, cs, len(data), case["codec"], max(len(data), 1))
    assert (out == data).all()


@pytest.mark.parametrize("case", G.chunk_cases(), ids=lambda c: c["key"])
def test_chunk_loop_vs_golden(torch_cuda, case):
    data = G.inp(case["input"])
    packed, cs = L.compress_chunks(data, case["codec"], case["chunk"], level=case["level"])
    assert (cs == G.arrays()[case["key"] + "/csizes"]).all()
    assert len(packed) == case["packed_bytes"] and G.sha(packed) == case["packed_sha256"]
    out = L.decompress_chunks(packed, cs, len(data), case["codec"], case["chunk"])
    assert (out == data).all()


@pytest.mark.parametrize("big", G.manifest()["large"], ids=lambda b: f"{b['corpus']}-{b['codec']}-{b['chunk']}")
def test_large_device_resident_vs_reference_digest(torch_cuda, big):
    torch = torch_cuda
    data = L.datagen(big["corpus"], big["size"], seed=big["seed"])
    assert G.sha(data) == big["input_sha256"]
    n = len(data)
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
    d_in[:n].copy_(torch.from_numpy(data))
    dc = L.DeviceCodec(big["codec"], n, big["chunk"])
    dc.compress(d_in)
    dc.decompress()
    torch.cuda.synchronize()
    total = dc.packed_total()
    assert total == big["packed_bytes"]
    assert G.sha(dc.packed[:total].cpu().numpy()) == big["packed_sha256"]
    assert G.sha(dc.csizes.cpu().numpy().astype(np.uint64)) == big["csizes_sha256"]
    assert (dc.status.cpu().numpy() >= 0).all()
    assert torch.equal(dc.out[:n], d_in[:n])


def _fullsize():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")) as f:
        return json.load(f)


def _per_gpu_sizes():
    """the 1-GPU workloads and, of the multi-GPU corpora, the first and the last share (offset != 0: the bytes
    rank r compresses); whole multi-GiB corpora: test_gpu_rows.py"""
    out = []
    for b in _fullsize():
        if "shares" in b:
            continue
        if b.get("offset", 0) and b["offset"] + b["size"] < max(e.get("offset", 0) + e["size"] for e in _fullsize()
                                                                 if (e["corpus"], e["codec"], e["chunk"]) ==
                                                                 (b["corpus"], b["codec"], b["chunk"]) and "shares" not in e):
            continue
        out.append(b)
    return out


@pytest.mark.parametrize("big", _per_gpu_sizes(),
                         ids=lambda b: f"{b['corpus']}{b['size'] >> 20}m@{b.get('offset', 0) >> 20}-{b['codec']}{b['level']}-b{b['chunk'] >> 10}")
def test_full_size_vs_reference_digest(torch_cuda, big):
    """BASELINE sizes (1 GiB per GPU): the whole packed stream and every compr_size equal the
    reference chunk loop's (sha256 from tests/golden/make_fullsize.py), plus the size-independent
    properties -- decode(encode(x)) == x, sum of chunk sizes == packed total, chunk sizes within
    the codec bound."""
    torch = torch_cuda
    n, chunk = big["size"], big["chunk"]
    data = L.datagen(big["corpus"], n, seed=big["seed"], offset=big.get("offset", 0))
    assert G.sha(data) == big["input_sha256"]
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
    d_in[:n].copy_(torch.from_numpy(data))
    del data
    dc = L.DeviceCodec(big["codec"], n, chunk, level=big["level"])
    dc.compress(d_in)
    dc.decompress()
    torch.cuda.synchronize()
    cs = dc.csizes.cpu().numpy().astype(np.uint64)
    total = dc.packed_total()
    assert int(dc.offsets[-1].item()) == int(cs.sum()) == total == big["packed_bytes"]
    bound = {"lz4": chunk + chunk // 255 + 16, "lz4fast": chunk + chunk // 255 + 16, "snappy": 32 + chunk + chunk // 6,
             "zstd": chunk + (chunk >> 8) + (((128 << 10) - chunk) >> 11 if chunk < (128 << 10) else 0)}[big["codec"]]
    assert (cs <= bound).all() and (cs > 0).all()
    assert G.sha(cs.astype("<u8")) == big["csizes_sha256"]
    assert G.sha(dc.packed[:total].cpu().numpy()) == big["packed_sha256"]
    assert (dc.status.cpu().numpy() == chunk).all()
    assert torch.equal(dc.out[:n], d_in[:n])


@pytest.mark.parametrize("bad", G.manifest()["malformed"], ids=lambda b: f"{b['codec']}-{b['name']}")
def test_malformed_streams_rejected_like_reference(torch_cuda, bad):
    torch = torch_cuda
    v = G.arrays()[bad["key"]]
    cap = bad["cap"]
    packed = torch.zeros(len(v) + 256, dtype=torch.uint8, device="cuda")
    packed[: len(v)].copy_(torch.from_numpy(v.copy()))
    dc = L.DeviceCodec(bad["codec"], cap, cap)
    cs = torch.tensor([len(v)], dtype=torch.int32, device="cuda")
    if len(v) == cap:
        pytest.skip("would be treated as a raw-stored chunk")
    dc.decompress(packed=packed, csizes=cs)
    torch.cuda.synchronize()
    st = int(dc.status[0].item())
    if bad["codec"] == "snappy" and bad["ok"]:
        assert st == 5000            # the valid stream decodes to its 5000 bytes
    else:
        assert (st >= 0) == bad["ok"], st


def test_lzbench_per_chunk_rows(torch_cuda):
    """The compressor_desc_t rows called exactly as lzbench_compress/_decompress do."""
    lib = L.lib()
    data = G.inp("text")[:65536].copy()
    for codec, init, comp, dec in (("lz4", "lzbench_hip_lz4_init", "lzbench_hip_lz4_compress", "lzbench_hip_lz4_decompress"),
                                   ("snappy", "lzbench_hip_snappy_init", "lzbench_hip_snappy_compress",
                                    "lzbench_hip_snappy_decompress")):
        wm = getattr(lib, init)(65536, 0, 1)
        assert wm
        out = np.zeros(L.get_compress_bound(65536), np.uint8)
        clen = getattr(lib, comp)(data.ctypes.data, 65536, out.ctypes.data, len(out), 0, 0, wm)
        exp = O.lz4_compress(data) if codec == "lz4" else O.snappy_compress(data)
        assert clen == len(exp) and out[:clen].tobytes() == exp
        back = np.zeros(65536 + 64, np.uint8)
        dlen = getattr(lib, dec)(out.ctypes.data, clen, back.ctypes.data, 65536, 0, 0, wm)
        assert dlen == 65536 and (back[:65536] == data).all()
        lib.lzbench_hip_deinit(wm)
    wm = lib.lzbench_hip_memcpy_init(65536, 0, 1)
    out = np.zeros(65536, np.uint8)
    assert lib.lzbench_hip_memcpy(data.ctypes.data, 65536, out.ctypes.data, 65536, 0, 0, wm) == 65536
    assert (out == data).all()
    lib.lzbench_hip_deinit(wm)


def test_batched_rows_multi_file_chunk_list(torch_cuda):
    """lzbench's chunk list over several files (lzbench.cpp:366-373): ragged tails per file."""
    files = [G.inp("text")[:150_000], G.inp("json")[:70_001], G.inp("runs")[:65536], G.inp("zeros")[:5]]
    chunk = 65536
    data = np.concatenate(files)
    sizes = np.concatenate([L.chunk_sizes_for(len(f), chunk) for f in files])
    for codec in ("lz4", "snappy"):
        packed, cs = L.compress_chunks(data, codec, chunk, chunk_sizes=sizes)
        exp_packed, exp_cs = [], []
        for f in files:
            p, c = O.compress_chunks(f.copy(), codec, chunk)
            exp_packed.append(p)
            exp_cs.append(c)
        assert (cs == np.concatenate(exp_cs)).all()
        assert (packed == np.concatenate(exp_packed)).all()
        out = L.decompress_chunks(packed, cs, len(data), codec, chunk, chunk_sizes=sizes)
        assert (out == data).all()


@pytest.mark.parametrize("acc", [1, 2, 3, 5, 17, 99])
def test_lz4fast_levels(torch_cuda, acc):
    data = L.datagen("mixed", 8 << 20, seed=3)
    name = "lz4fast" if acc > 1 else "lz4"
    packed, cs = L.compress_chunks(data, name, 65536, level=acc)
    ep, ec = O.compress_chunks(data, name, 65536, acc)
    assert (cs == ec).all() and (packed == ep).all()


def _runs(n, seed):
    rng = np.random.default_rng(seed)
    return np.repeat(rng.integers(0, 3, n // 4 + 16, dtype=np.uint8), rng.integers(1, 40, n // 4 + 16))[:n].copy()


@pytest.mark.parametrize("acc", [2, 3, 4, 7, 64, 65, 200])
@pytest.mark.parametrize("kind", ["text", "json", "binary", "random", "runs"])
def test_lz4fast_pattern_batches(torch_cuda, acc, kind):
    """Probe-pattern run batches (acc > 1) across corpora, byU16 and byU32 tables, ragged tails
    and tiny chunks (where the tail switches to stride batches)."""
    n = 3 << 20
    data = _runs(n, 4) if kind == "runs" else L.datagen(kind, n, seed=11)
    for chunk in (65536, 1 << 20, 4099, 65547):
        packed, cs = L.compress_chunks(data, "lz4fast", chunk, level=acc)
        ep, ec = O.compress_chunks(data, "lz4fast", chunk, acc)
        assert (cs == ec).all() and (packed == ep).all(), (kind, acc, chunk)
    out = L.decompress_chunks(packed, cs, len(data), "lz4", chunk)
    assert (out == data).all()


def test_unaligned_chunk_bases(torch_cuda):
    """Chunk sizes that are not multiples of 4 put chunk starts at every byte alignment."""
    data = L.datagen("json", 1_000_003, seed=9)
    for codec in ("lz4", "snappy"):
        for chunk in (65533, 70001, 4099):
            packed, cs = L.compress_chunks(data, codec, chunk)
            ep, ec = O.compress_chunks(data, codec, chunk)
            assert (cs == ec).all() and (packed == ep).all(), (codec, chunk)
            out = L.decompress_chunks(packed, cs, len(data), codec, chunk)
            assert (out == data).all()
