"""CPU: the C-ABI library loads and exports every symbol include/lzbench_hip.h declares; host
logic of the Python mirror; the product never touches the oracle.  No GPU compute calls."""
import os
import re
import subprocess

import numpy as np
import pytest

import lzbench_amd as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lzbench_hip.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lz[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_entry_points():
    names = header_functions()
    for must in ("lzbench_hip_lz4_compress", "lzbench_hip_lz4_decompress", "lzbench_hip_snappy_compress",
                 "lzbench_hip_snappy_decompress", "lzbench_hip_compress_batch", "lzbench_hip_decompress_batch",
                 "lzh_compress_async", "lzh_decompress_async"):
        assert must in names


def test_library_exports_every_header_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [f for f in header_functions() if f not in exported]
    assert not missing, missing


def test_python_signatures_cover_header_and_load():
    lib = L.lib()                      # loads the .so and binds every signature
    assert set(header_functions()) == set(L.SIGNATURES)
    assert b"gfx950" in lib.lzh_version()


def test_size_helpers():
    lib = L.lib()
    assert lib.lzh_num_chunks(1 << 30, 65536) == 16384
    assert lib.lzh_num_chunks(65537, 65536) == 2
    assert lib.lzh_num_chunks(0, 65536) == 1
    s = lib.lzh_stage_stride(0, 65536)
    assert s % 256 == 0 and s >= 65536 + 65536 // 255 + 16       # >= LZ4_compressBound
    assert lib.lzh_stage_stride(1, 65536) >= 32 + 65536 + 65536 // 6  # >= MaxCompressedLength
    assert lib.lzh_compress_temp_bytes(0, 1 << 30, 65536) >= 16384 * s
    assert lib.lzh_max_packed_bytes(0, 1 << 20, 65536) >= 16 * (65536 + 65536 // 255 + 16)


@pytest.mark.parametrize("chunk", [1024, 4096, 16384, 131072])
def test_zstd_decode_temp_stays_proportionate(chunk):
    """zstd decode temp per GiB: below 16 KiB chunks the split decoder's per-frame layout (two block slots
    and 2 x chunk of sequence records, ~20x the input at -b1) is not reserved -- those frames decode in
    the one-wave kernel -- so -b1 / -b4 need only the offsets; from 16 KiB on the layout costs a few x."""
    lib = L.lib()
    n = 1 << 30
    t = lib.lzh_decompress_temp_bytes(3, n, chunk)
    k = lib.lzh_num_chunks(n, chunk)
    if chunk < 16384:
        assert t <= 8 * (k + 1) + 1024
    else:
        assert t <= 4 * n


def test_comp_desc_table_mirrors_lzbench():
    assert L.COMP_DESC[0].name == "memcpy"                   # lzbench.cpp:609, :695
    assert L.find_compressor("lz4").name == "hip_lz4"
    assert L.find_compressor("snappy").name == "hip_snappy"
    assert (L.find_compressor("lz4fast").first_level, L.find_compressor("lz4fast").last_level) == (1, 99)
    with pytest.raises(KeyError):
        L.find_compressor("zling")
    syms = set(L.SIGNATURES)
    for d in L.COMP_DESC[1:]:
        for f in (d.compress, d.decompress, d.init, d.deinit, d.compress_batch, d.decompress_batch):
            assert f in syms


def test_chunk_list_like_lzbench():
    cs = L.chunk_sizes_for(200_000, 65536)                   # lzbench.cpp:366-373
    assert cs.tolist() == [65536, 65536, 65536, 3392]
    assert L.chunk_sizes_for(131072, 65536).tolist() == [65536, 65536]
    assert L.get_compress_bound(600) == 600 + 100 + 16384


def test_datagen_deterministic_and_segmented():
    a = L.datagen("text", 40 << 20, seed=3)
    b = L.datagen("text", 40 << 20, seed=3)
    assert (a == b).all()
    c = L.datagen("text", 20 << 20, seed=3)                   # same prefix regardless of length
    assert (a[: 20 << 20] == c).all()
    assert set(np.unique(L.datagen("text", 1 << 16, seed=1))) <= set(b"abcdefghijklmnopqrstuvwxyz \n")


def test_product_sources_never_reference_the_oracle():
    for d, _, files in os.walk(os.path.join(ROOT, "lzbench_amd")):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".c", ".h")):
                txt = open(os.path.join(d, f)).read()
                for bad in ("liboracle", "libref", "oracle_lib", "import oracle", "oracle/"):
                    assert bad not in txt, (f, bad)


def _plan(ngpus, n, chunk, codec=0):
    out = (C_U64 * 80)()
    m = L.lib().lzh_debug_plan(ngpus, n, chunk, codec, out, 80)
    v = [int(x) for x in out[:m]]
    k, sbk, nsb, G, sb_in, sb_packed, sb_temp = v[:7]
    return dict(k=k, sbk=sbk, nsb=nsb, G=G, sb_in=sb_in, sb_packed=sb_packed, sb_temp=sb_temp, slots=v[7:])


import ctypes as _C  # noqa: E402
C_U64 = _C.c_uint64


@pytest.mark.parametrize("ngpus", [1, 2, 3, 8, 64])
@pytest.mark.parametrize("n,chunk", [(0, 65536), (1, 65536), (65537, 65536), (1 << 30, 65536), (3 << 20, 1_790_000_000),
                                     ((300 << 20) + 77, 65536), (1 << 40, 65536), (8 << 30, 1 << 20), (12345, 100)])
def test_batched_row_plan_arithmetic(ngpus, n, chunk):
    """api.cpp make_plan (the batched rows' sharding, host arithmetic only): every chunk in exactly one
    sub-batch, sub-batches dealt round-robin (shard slot counts differ by at most one), a sub-batch's
    buffers sized from the bytes actually present (one chunk of lzbench's default 1.79 GB chunk size
    over a 3 MiB file must not size 1024 chunks: round 1's 1 TB hipMalloc), and no shard's buffers
    exceed its share of the input by more than one sub-batch."""
    p = _plan(ngpus, n, chunk)
    chunk = max(min(chunk, n), 1)                  # (api.cpp row_chunk)
    k = max(1, -(-n // chunk))
    assert p["k"] == k
    assert p["nsb"] * p["sbk"] >= k > (p["nsb"] - 1) * p["sbk"]
    assert p["G"] == min(ngpus, k, p["nsb"]) and len(p["slots"]) == p["G"]
    assert sum(p["slots"]) == p["nsb"] and max(p["slots"]) - min(p["slots"]) <= 1
    assert p["sb_in"] == min(n, p["sbk"] * chunk)
    assert p["sb_packed"] >= p["sb_in"] and p["sb_packed"] % 256 == 0
    assert p["sb_packed"] <= p["sb_in"] + p["sbk"] * (chunk // 6 + 300) + 4096
    assert max(p["slots"]) * p["sb_in"] <= -(-n // p["G"]) + p["sb_in"]
    if n < (64 << 20):
        assert p["sb_temp"] < (256 << 20)


@pytest.mark.parametrize("nsb,seed", [(1, 0), (2, 1), (7, 2), (16, 3), (64, 4)])
def test_gather_places_each_sub_batch_as_soon_as_its_offset_is_known(nsb, seed):
    """api.cpp GatherOrder (the batched rows' host gather, polled over every shard's sub-batches):
    whatever order the sub-batches finish in, each is copied out at the exclusive prefix sum of the
    packed sizes (lzbench.cpp:266-298 packing), in chunk order, and at the first completion after
    which it and everything before it are known -- never later."""
    rng = np.random.default_rng(seed)
    order = rng.permutation(nsb).astype(np.uint64)
    sizes = rng.integers(0, 1 << 27, nsb).astype(np.uint64)
    placed = np.zeros(3 * nsb, np.uint64)
    lib = L.lib()
    m = lib.lzh_debug_gather_order(nsb, order.ctypes.data, sizes.ctypes.data, placed.ctypes.data)
    assert m == nsb
    pl = placed.reshape(-1, 3)
    assert pl[:, 0].tolist() == list(range(nsb))
    assert pl[:, 1].tolist() == np.concatenate([[0], np.cumsum(sizes)[:-1]]).tolist()
    pos = np.empty(nsb, np.int64)
    pos[order.astype(np.int64)] = np.arange(nsb)
    assert pl[:, 2].tolist() == np.maximum.accumulate(pos).tolist()


def test_level_supported():
    lib = L.lib()
    assert lib.lzh_level_supported(3, 1, 1 << 20) == 1          # zstd 1: fast strategy at every size
    assert lib.lzh_level_supported(3, 2, 131072) == 1           # zstd 2: fast up to 256 KiB chunks
    assert lib.lzh_level_supported(3, 2, 1 << 20) == 0          # ... double-fast above (clevels.h)
    assert lib.lzh_level_supported(3, 3, 65536) == 0
    assert lib.lzh_level_supported(3, -5, 1 << 20) == 1
    assert lib.lzh_level_supported(4, 0x88, 65536) == 0 and lib.lzh_level_supported(4, 0x74, 65536) == 1
    assert lib.lzh_level_supported(4, 0x80, 65536) == 1 and lib.lzh_level_supported(4, 0x3F4, 1 << 20) == 1
    assert lib.lzh_level_supported(5, 6, 65536) == 0 and lib.lzh_level_supported(0, 1, 65536) == 1
