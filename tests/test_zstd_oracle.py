"""zstd compression restatement (oracle/zstd1_oracle.c) pinned to the reference: every digest of
tests/golden/zstd_cgolden.json (made by the reference build through lzbench's chunk loop) is
reproduced by the restatement, and on fresh inputs the restatement equals the reference build
(oracle/_ref, where present) frame for frame.  CPU only."""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O
import lzbench_amd as L

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def cgolden():
    with open(os.path.join(GOLD, "zstd_cgolden.json")) as f:
        return json.load(f)["cases"]


def corpus(kind, n, seed):
    if kind == "zeros":
        d = np.zeros(n, np.uint8)
        d[::4099] = 7
        return d
    if kind == "runs":
        rng = np.random.default_rng(seed)
        return np.repeat(rng.integers(0, 4, n // 8 + 16, dtype=np.uint8),
                         rng.integers(1, 300, n // 8 + 16))[:n].copy()
    return L.datagen(kind, n, seed)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.parametrize("case", cgolden(), ids=lambda c: f"{c['corpus']}-{c['n']}-b{c['chunk'] >> 10}-l{c['level']}")
def test_restatement_reproduces_reference_digest(case):
    data = corpus(case["corpus"], case["n"], case["seed"])
    assert sha(data) == case["input_sha256"]
    packed, cs = O.compress_chunks(data, "zstd", case["chunk"], case["level"], use_ref=False)
    assert len(packed) == case["packed_bytes"]
    assert sha(cs.astype("<u8")) == case["csizes_sha256"]
    assert sha(packed) == case["packed_sha256"]


@pytest.mark.parametrize("level", [1, -1, -4])
def test_restatement_equals_reference_on_random_slices(level):
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    rng = np.random.default_rng(level + 100)
    src = np.concatenate([L.datagen("mixed", 1 << 21, seed=3), corpus("runs", 1 << 20, 4),
                          rng.integers(0, 3, 1 << 19, dtype=np.uint8)])
    for _ in range(12):
        n = int(rng.integers(1, 700_000))
        off = int(rng.integers(0, len(src) - n))
        chunk = int(rng.choice([65536, 131072, 262144, 524288, 1 << 20]))
        data = src[off:off + n].copy()
        a, ca = O.compress_chunks(data, "zstd", chunk, level, use_ref=False)
        b, cb = O.compress_chunks(data, "zstd", chunk, level, use_ref=True)
        assert (ca == cb).all() and a.tobytes() == b.tobytes(), (n, chunk, level)



def mixed_chunk_11359():
    """chunk 11359 (128 KiB) of the 4 GiB seed-12345 mixed corpus (config 5): its literal histogram has nine
    symbols of count 164, which HUF_sort's bucket loop quick-sorts (huf_compress.c:585-592: the loop starts at
    RANK_POSITION_DISTINCT_COUNT_CUTOFF = 158 + BIT_highbit32(158) = 165, and region 165 holds the symbols of
    count 164); the quicksort reorders the tie, and two of the nine straddle the depth-9 / depth-10 boundary"""
    ck, i = 131072, 11359
    seg = (i * ck) // (16 << 20) * (16 << 20)
    d = L.datagen("mixed", 32 << 20, seed=12345, offset=seg)
    return np.ascontiguousarray(d[i * ck - seg:(i + 1) * ck - seg])


@pytest.mark.skipif(not O.have_ref(), reason="needs oracle/_ref (the reference build)")
def test_huffman_sort_cutoff_equals_reference():
    """The restatement's HUF_sort cutoff is the macro's value (165), not its comment's (166): found by the 4 GiB
    config-5 digest (tests/test_gpu_rows.py), where this chunk alone came out with the same size and different
    Huffman code lengths for two symbols of equal count."""
    d = mixed_chunk_11359()
    rp, rcs = O.compress_chunks(d, "zstd", 131072, 1, use_ref=True)
    op, ocs = O.compress_chunks(d, "zstd", 131072, 1, use_ref=False)
    assert (rcs == ocs).all() and len(rp) == len(op) and (rp == op).all()
