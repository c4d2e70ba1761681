#!/usr/bin/env python3
"""tests/golden/make_zstd_cgolden.py -- golden digests for zstd COMPRESSION (the hip_zstd row):
the reference zstd 1.5.2 build (oracle/_ref/libref.so, lzbench's zstd row semantics:
ZSTD_getParams(level, chunk, 0) + contentSizeFlag + ZSTD_compress_advanced, compressors.cpp:
1745-1770) run through lzbench's chunk loop (lzbench.cpp:266-298: raw-store rule, contiguous
packing) on the repo's deterministic corpora.  Stored: sha256 of the packed stream and of the
compr_sizes (little-endian u64), plus the packed byte count; inputs regenerate from the seeds.

Covers the fast-strategy levels (zstd 1 and 2 where fast, zstd_fast -1..-5), single-block frames
(-b64, -b128), multi-block frames with Huffman-table repeats and RLE blocks (-b256 .. -b1024,
the latter beyond the 512 KiB window), raw chunks, tiny and ragged tails.
Run from the repo root:  python tests/golden/make_zstd_cgolden.py"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import lzbench_amd as L  # noqa: E402
import oracle_lib as O  # noqa: E402


def corpus(kind, n, seed):
    """Synthetic inputs: lzh_datagen corpora, plus zero runs with sparse literals and short runs."""
    if kind == "zeros":
        d = np.zeros(n, np.uint8)
        d[::4099] = 7
        return d
    if kind == "runs":
        rng = np.random.default_rng(seed)
        return np.repeat(rng.integers(0, 4, n // 8 + 16, dtype=np.uint8),
                         rng.integers(1, 300, n // 8 + 16))[:n].copy()
    return L.datagen(kind, n, seed)


CASES = []
for kind in ("text", "json", "mixed", "binary", "random", "zeros", "runs"):
    for chunk in (65536, 131072, 262144, 524288):
        CASES.append((kind, 3 * chunk + 12345, chunk, 1))
for kind in ("text", "mixed", "runs"):
    CASES.append((kind, (1 << 21) + 77, 1 << 20, 1))     # frames larger than the 512 KiB window
    for level in (-1, -3, -5, 2):
        CASES.append((kind, 600_000, 131072, level))
for n in (1, 7, 8, 37, 63, 64, 255, 256, 1023, 1024, 16384, 16385, 65792, 65793):
    CASES.append(("text", n, 131072, 1))


def main():
    cases = []
    for kind, n, chunk, level in CASES:
        seed = 5
        data = corpus(kind, n, seed)
        packed, cs = O.compress_chunks(data, "zstd", chunk, level, use_ref=True)
        e = dict(corpus=kind, n=n, chunk=chunk, level=level, seed=seed,
                 input_sha256=hashlib.sha256(data.tobytes()).hexdigest(),
                 packed_sha256=hashlib.sha256(packed.tobytes()).hexdigest(),
                 csizes_sha256=hashlib.sha256(cs.astype("<u8").tobytes()).hexdigest(),
                 packed_bytes=int(len(packed)))
        cases.append(e)
        print(e["corpus"], n, chunk, level, len(packed), flush=True)
    with open(os.path.join(ROOT, "tests", "golden", "zstd_cgolden.json"), "w") as f:
        json.dump({"generator": "zstd 1.5.2 reference build (oracle/_ref), tests/golden/make_zstd_cgolden.py",
                   "version": int(O.ref().ref_zstd_version()), "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
