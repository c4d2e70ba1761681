"""GPU stress parity: the HIP compressors and decoders against the oracle on inputs built to
exercise the lane-parallel batch resolve -- many in-batch hash-slot collisions, immediate
re-test hits, matches that end inside / exactly at / past a 64-position batch, long and short
literal runs, and the switch between run batches and search batches.  Bit-exact bytes and sizes
for every chunk, and a round trip.  Run with -m gpu.

Inputs are seeded synthetic data (no reference fixture covers them: parity here is against the
oracle restatement, which tests/test_oracle.py pins to the reference's own outputs)."""
import numpy as np
import pytest

import oracle_lib as O
import lzbench_amd as L

pytestmark = pytest.mark.gpu

SIZE = 2 << 20


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    return torch


def _lowent(rng):
    """4-letter alphabet in random runs: dense matches, many equal 4-grams per batch."""
    vals = rng.integers(0, 4, SIZE // 3).astype(np.uint8) + ord("a")
    runs = rng.integers(1, 6, len(vals))
    return np.repeat(vals, runs)[:SIZE]


def _periodic(rng):
    """a random line repeated with sparse mutations: re-test hits, matches crossing batches."""
    out = np.empty(SIZE, np.uint8)
    pos = 0
    while pos < SIZE:
        period = int(rng.integers(3, 200))
        line = rng.integers(32, 127, period).astype(np.uint8)
        reps = int(rng.integers(2, 60))
        blk = np.tile(line, reps)
        mut = rng.random(len(blk)) < 0.01
        blk[mut] = rng.integers(32, 127, int(mut.sum())).astype(np.uint8)
        n = min(len(blk), SIZE - pos)
        out[pos:pos + n] = blk[:n]
        pos += n
    return out


def _tinyvocab(rng):
    """text from 12 short words: repeated 4-grams with different continuations (slot groups)."""
    words = [b"a ", b"an ", b"the ", b"then ", b"than ", b"at ", b"ate ", b"eat ", b"tea ", b"ten ", b"net ", b"\n"]
    idx = rng.integers(0, len(words), SIZE // 2)
    return np.frombuffer(b"".join(words[i] for i in idx), np.uint8)[:SIZE].copy()


def _mixed_stripes(rng):
    """compressible text, random bytes and zero runs in 3-17 KiB stripes: search batches, long
    literals, long matches and the run/search switches between them."""
    out = np.empty(SIZE, np.uint8)
    pos = 0
    while pos < SIZE:
        n = min(int(rng.integers(3 << 10, 17 << 10)), SIZE - pos)
        kind = int(rng.integers(0, 3))
        if kind == 0:
            out[pos:pos + n] = L.datagen("text", n, seed=int(rng.integers(1, 1 << 30)))
        elif kind == 1:
            out[pos:pos + n] = rng.integers(0, 256, n).astype(np.uint8)
        else:
            out[pos:pos + n] = 0
        pos += n
    return out


GENS = {"lowent": _lowent, "periodic": _periodic, "tinyvocab": _tinyvocab, "stripes": _mixed_stripes}
CONFIGS = [("lz4", 65536, 1), ("lz4", 131072, 1), ("lz4fast", 65536, 2), ("snappy", 65536, 0), ("snappy", 262144, 0)]


@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("gen", sorted(GENS))
@pytest.mark.parametrize("cfg", CONFIGS, ids=lambda c: f"{c[0]}-b{c[1] >> 10}-l{c[2]}")
def test_stress_vs_oracle(torch_cuda, gen, seed, cfg):
    codec, chunk, level = cfg
    data = GENS[gen](np.random.default_rng(1000 * seed + len(gen)))
    packed, cs = L.compress_chunks(data, codec, chunk, level)
    exp_packed, exp_cs = O.compress_chunks(data, codec, chunk, level)
    bad = np.nonzero(cs != exp_cs)[0]
    assert len(bad) == 0, f"chunk sizes differ first at chunk {bad[:4]}: {cs[bad[:4]]} vs {exp_cs[bad[:4]]}"
    assert len(packed) == len(exp_packed) and (packed == exp_packed).all(), "packed bytes differ"
    out = L.decompress_chunks(packed, cs, len(data), codec, chunk)
    assert (out == data).all()


def _copies_chunks():
    """64 KiB chunks of random bytes, each with k copies of earlier 16-byte blocks (about one sequence per
    copy: no other 4-byte repeats) spaced s bytes apart: record counts around the emission kernels' 64-record
    groups and their one-group-ahead loads (k = 0 .. 300), input spans that fit the group's LDS copy (s = 20)
    and spans that do not (s = 200: the record-by-record path)."""
    rng = np.random.default_rng(4242)
    chunks = []
    for s in (20, 200):
        for k in (0, 1, 2, 63, 64, 65, 127, 128, 129, 191, 192, 193, 256, 300):
            c = rng.integers(0, 256, 65536).astype(np.uint8)
            for i in range(k):
                pos = 1024 + i * s
                src = int(rng.integers(0, pos - 32))
                c[pos:pos + 16] = c[src:src + 16]
            chunks.append(c)
    return np.concatenate(chunks)


@pytest.mark.parametrize("codec", ["lz4", "snappy"])
def test_emission_group_boundaries(torch_cuda, codec):
    data = _copies_chunks()
    packed, cs = L.compress_chunks(data, codec, 65536, 1 if codec == "lz4" else 0)
    exp_packed, exp_cs = O.compress_chunks(data, codec, 65536, 1 if codec == "lz4" else 0)
    bad = np.nonzero(cs != exp_cs)[0]
    assert len(bad) == 0, f"chunk sizes differ first at chunk {bad[:4]}: {cs[bad[:4]]} vs {exp_cs[bad[:4]]}"
    assert len(packed) == len(exp_packed) and (packed == exp_packed).all(), "packed bytes differ"
    out = L.decompress_chunks(packed, cs, len(data), codec, 65536)
    assert (out == data).all()
