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
