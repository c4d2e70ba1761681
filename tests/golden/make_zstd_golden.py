"""tests/golden/make_zstd_golden.py -- zstd 1.5.2 frames made by the REFERENCE build
(oracle/_ref/libref.so, lzbench's zstd row semantics: ZSTD_getParams(level, chunk, 0),
contentSizeFlag = 1, ZSTD_compress_advanced; compressors.cpp:1745-1765) for the GPU decoder's
golden tests.  Inputs are the repo's deterministic synthetic corpora (lzh_datagen), so only the
frames, their per-chunk sizes and the input digests are stored.  Run from the repo root:
    python tests/golden/make_zstd_golden.py"""
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

# (name, corpus, n, chunk, level): compressed, raw, RLE and multi-block frames, tiny inputs
CASES = [
    ("text_b128_l1", "text", 300_000, 131072, 1),
    ("json_b64_l1", "json", 200_000, 65536, 1),
    ("binary_b256_l3", "binary", 100_003, 262144, 3),
    ("random_b128_l1", "random", 40_000, 131072, 1),
    ("zeros_b128_l1", "zeros", 131072 + 5000, 131072, 1),
    ("text_b128_l19", "text", 131072, 131072, 19),
    ("text_tiny_l1", "text", 37, 131072, 1),
    ("json_b1024_l1", "json", 1 << 20, 1 << 20, 1),
]


def corpus(kind, n, seed=5):
    if kind == "zeros":
        d = np.zeros(n, np.uint8)
        d[::4099] = 7                                   # a few literals between long runs
        return d
    return L.datagen(kind, n, seed)


def main():
    arrays, cases = {}, []
    for name, kind, n, chunk, level in CASES:
        data = corpus(kind, n)
        packed, cs = O.compress_chunks(data, "zstd", chunk, level)
        arrays[f"{name}/packed"] = packed
        arrays[f"{name}/csizes"] = cs.astype(np.uint64)
        cases.append(dict(name=name, corpus=kind, n=n, chunk=chunk, level=level, seed=5,
                          input_sha256=hashlib.sha256(data.tobytes()).hexdigest()))
    out = os.path.join(ROOT, "tests", "golden")
    np.savez_compressed(os.path.join(out, "zstd_golden.npz"), **arrays)
    with open(os.path.join(out, "zstd_manifest.json"), "w") as f:
        json.dump({"generator": "zstd 1.5.2 reference build (oracle/_ref)", "version": int(O.ref().ref_zstd_version()),
                   "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
