"""CPU: the oracle restatement (oracle/*.c) against the reference's own outputs (tests/golden),
and lzbench chunk-loop semantics.  No GPU needed."""
import numpy as np
import pytest

import golden_data as G
import oracle_lib as O
import lzbench_amd as L


@pytest.mark.parametrize("case", G.block_cases(), ids=lambda c: c["key"])
def test_block_compress_matches_reference(case):
    data = G.inp(case["input"])[: case["n"]].copy()
    got = O.lz4_compress(data, case["acc"]) if case["codec"] == "lz4" else O.snappy_compress(data)
    assert G.check_block(case, got)


@pytest.mark.parametrize("case", G.block_cases(), ids=lambda c: c["key"])
def test_block_roundtrip(case):
    data = G.inp(case["input"])[: case["n"]].copy()
    lib = O.oracle()
    out = np.zeros(len(data) + 64, np.uint8)
    if case["codec"] == "lz4":
        comp = np.frombuffer(O.lz4_compress(data, case["acc"]), np.uint8).copy()
        r = lib.oracle_lz4_decompress_safe(comp.ctypes.data, len(comp), out.ctypes.data, len(data))
    else:
        comp = np.frombuffer(O.snappy_compress(data), np.uint8).copy()
        r = lib.oracle_snappy_uncompress(comp.ctypes.data, len(comp), out.ctypes.data, len(data))
    assert r == len(data)
    assert (out[: len(data)] == data).all()


@pytest.mark.parametrize("case", G.chunk_cases(), ids=lambda c: c["key"])
def test_chunk_loop_matches_reference(case):
    data = G.inp(case["input"])
    packed, cs = O.compress_chunks(data, case["codec"], case["chunk"], case["level"])
    assert (cs == G.arrays()[case["key"] + "/csizes"]).all()
    assert len(packed) == case["packed_bytes"] and G.sha(packed) == case["packed_sha256"]
    r, out = O.decompress_chunks(packed, cs, len(data), case["codec"], case["chunk"])
    assert r == len(data) and (out == data).all()


def test_raw_store_rule():
    """lzbench.cpp:284-288: an expanded chunk stays compressed, a chunk whose compressed size
    equals its size would be stored raw (compr_size == part) and decoded by memcpy."""
    data = L.datagen("random", 131072, seed=5)
    packed, cs = O.compress_chunks(data, "lz4", 65536)
    assert (cs > 65536).all()                    # lz4 expands random data: kept compressed
    r, out = O.decompress_chunks(packed, cs, len(data), "lz4", 65536)
    assert r == len(data) and (out == data).all()


@pytest.mark.parametrize("bad", G.manifest()["malformed"], ids=lambda b: f"{b['codec']}-{b['name']}")
def test_malformed_verdicts(bad):
    v = G.arrays()[bad["key"]].copy()
    lib = O.oracle()
    out = np.zeros((1 << 20) + 64, np.uint8)
    if bad["codec"] == "lz4":
        r = lib.oracle_lz4_decompress_safe(v.ctypes.data, len(v), out.ctypes.data, bad["cap"])
        assert (r >= 0) == bad["ok"]
    else:
        r = lib.oracle_snappy_uncompress(v.ctypes.data, len(v), out.ctypes.data, 1 << 20)
        assert (r >= 0) == bad["ok"]


@pytest.mark.parametrize("big", [b for b in G.manifest()["large"] if b["size"] <= (64 << 20)],
                         ids=lambda b: f"{b['corpus']}-{b['codec']}-{b['chunk']}")
def test_large_digests(big):
    data = L.datagen(big["corpus"], big["size"], seed=big["seed"])
    assert G.sha(data) == big["input_sha256"], "datagen output changed: regenerate tests/golden"
    packed, cs = O.compress_chunks(data, big["codec"], big["chunk"], 1, threads=8)
    assert len(packed) == big["packed_bytes"]
    assert G.sha(packed) == big["packed_sha256"] and G.sha(cs) == big["csizes_sha256"]


@pytest.mark.skipif(not O.have_ref(), reason="reference build (oracle/_ref) not present")
def test_oracle_equals_reference_fresh_random():
    """Beyond the stored vectors: fresh seeded inputs of many sizes, oracle vs the compiled reference."""
    rng = np.random.default_rng(99)
    for trial in range(40):
        n = int(rng.integers(0, 200_000))
        kind = ["text", "json", "binary", "random"][trial % 4]
        data = L.datagen(kind, n, seed=1000 + trial) if n else np.zeros(0, np.uint8)
        for codec, chunk in (("lz4", 65536), ("lz4", 131072), ("snappy", 65536), ("snappy", 262144)):
            if n == 0:
                continue
            a = O.compress_chunks(data, codec, chunk)
            b = O.compress_chunks(data, codec, chunk, use_ref=True)
            assert (a[1] == b[1]).all() and (a[0] == b[0]).all(), (trial, n, kind, codec, chunk)


@pytest.mark.skipif(not O.have_ref(), reason="reference build (oracle/_ref) not present")
@pytest.mark.parametrize("gen", ["lowent", "periodic", "tinyvocab", "stripes"])
@pytest.mark.parametrize("cfg", [("lz4", 65536, 1), ("lz4", 131072, 1), ("lz4fast", 65536, 2), ("snappy", 65536, 0),
                                 ("snappy", 262144, 0)], ids=lambda c: f"{c[0]}-b{c[1] >> 10}-l{c[2]}")
def test_oracle_matches_reference_on_stress_inputs(gen, cfg):
    """the GPU stress inputs (tests/test_gpu_stress.py) through the restatement and the reference build"""
    import test_gpu_stress as S
    codec, chunk, level = cfg
    data = S.GENS[gen](np.random.default_rng(1000 + len(gen)))
    p, cs = O.compress_chunks(data, codec, chunk, level)
    rp, rcs = O.compress_chunks(data, codec, chunk, level, use_ref=True)
    assert (cs == rcs).all() and len(p) == len(rp) and (p == rp).all()
