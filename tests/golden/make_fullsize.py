#!/usr/bin/env python3
"""tests/golden/make_fullsize.py -- sha256 digests of the REFERENCE chunk loop at BASELINE.json's
full sizes (1 GiB per GPU), so the GPU output of the bench workloads is compared whole, byte for
byte, not by sampled chunks.

Run in the build container (needs oracle/_ref/libref.so: lz4 1.9.3 / snappy 1.1.8 / zstd 1.5.2
compiled from /root/reference by `make -C oracle ref`).  Inputs are regenerated deterministically
by lzbench_amd.datagen (seed 12345 = bench.py's rank-0 input), so only digests are stored.

Writes fullsize.json: [{corpus, size, seed, codec, chunk, level, input_sha256, packed_sha256,
csizes_sha256, packed_bytes}], csizes hashed as little-endian u64 (lzbench's size_t array).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import lzbench_amd as L          # noqa: E402  (datagen only)
import oracle_lib as O           # noqa: E402

# (corpus, codec, chunk, level, size): the north star, config 3 at 1 GiB, config 4's per-GPU share,
# config 5's codec at its chunk size on a 1 GiB per-GPU share; then the other sweep lines of
# tools/config_sweep.sh at their exact sizes: config 2 (256 MiB text), config 5's 8-GPU per-GPU
# share (512 MiB mixed), lz4fast,3 on the north-star input
WORKLOADS = [
    ("text", "lz4", 65536, 1, 1 << 30),
    ("mixed", "snappy", 262144, 0, 1 << 30),
    ("json", "lz4", 65536, 1, 1 << 30),
    ("json", "snappy", 65536, 0, 1 << 30),
    ("mixed", "zstd", 131072, 1, 1 << 30),
    ("text", "lz4", 65536, 1, 256 << 20),
    ("mixed", "zstd", 131072, 1, 512 << 20),
    ("text", "lz4fast", 65536, 3, 1 << 30),
]
SEED = 12345
# multi-GPU workloads as one corpus cut into contiguous per-GPU shares (lzbench.cpp:366-373 cuts ONE
# file into one chunk list; rank r of N owns share r): (corpus, codec, chunk, level, share bytes,
# shares).  Each share is pinned on its own (offset = r x share: what rank r of bench.py compresses)
# and the whole corpus by the digest of the shares' packed streams / compr_sizes concatenated (what
# the host gather assembles): the north star at 1/2/4/8 GPUs (1 GiB of text per GPU), config 4
# (8 GiB JSON, lz4 and snappy -b64) and config 5 (4 GiB mixed, zstd-1 -b128, 512 MiB per GPU).
SHARED = [
    ("text", "lz4", 65536, 1, 1 << 30, 8),
    ("json", "lz4", 65536, 1, 1 << 30, 8),
    ("json", "snappy", 65536, 0, 1 << 30, 8),
    ("mixed", "zstd", 131072, 1, 512 << 20, 8),
]


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def entry_key(e):
    return (e["corpus"], e["codec"], e["chunk"], e["level"], e["size"], e.get("offset", 0))


def shared(out, path, only):
    """share and aggregate digests of SHARED (entries carry "offset"; aggregates of the first 2, 4 and
    all shares carry "shares": the whole corpus at 2, 4 and 8 GPUs)"""
    have = {entry_key(e) for e in out}
    for corpus, codec, chunk, level, share, nsh in SHARED:
        if only and codec not in only:
            continue
        prefixes = [m for m in (2, 4, 8) if m <= nsh]
        need = [(corpus, codec, chunk, level, share, r * share) for r in range(nsh)] + \
               [(corpus, codec, chunk, level, share * m, 0) for m in prefixes]
        if all(k in have for k in need):
            continue
        hp, hc, hin, tot = hashlib.sha256(), hashlib.sha256(), hashlib.sha256(), 0
        for r in range(nsh):
            data = L.datagen(corpus, share, seed=SEED, offset=r * share)
            packed, cs = O.compress_chunks(data, codec, chunk, level, use_ref=True, threads=8)
            hin.update(data.tobytes())
            hp.update(packed.tobytes())
            hc.update(cs.astype("<u8").tobytes())
            tot += len(packed)
            if (corpus, codec, chunk, level, share, r * share) not in have:
                e = {"corpus": corpus, "size": share, "offset": r * share, "seed": SEED, "codec": codec,
                     "chunk": chunk, "level": level, "input_sha256": sha(data), "packed_sha256": sha(packed),
                     "csizes_sha256": sha(cs.astype("<u8")), "packed_bytes": int(len(packed)),
                     "ratio_pct": round(100 * len(packed) / share, 3)}
                print(e, flush=True)
                out.append(e)
                have.add(entry_key(e))
            del data, packed, cs
            m = r + 1
            if m in prefixes and (corpus, codec, chunk, level, share * m, 0) not in have:
                e = {"corpus": corpus, "size": share * m, "offset": 0, "shares": m, "seed": SEED, "codec": codec,
                     "chunk": chunk, "level": level, "input_sha256": hin.copy().hexdigest(),
                     "packed_sha256": hp.copy().hexdigest(), "csizes_sha256": hc.copy().hexdigest(),
                     "packed_bytes": int(tot), "ratio_pct": round(100 * tot / (share * m), 3)}
                print(e, flush=True)
                out.append(e)
                have.add(entry_key(e))
            with open(path, "w") as f:
                json.dump(out, f, indent=1)


def main():
    if not O.have_ref():
        sys.exit("oracle/_ref/libref.so missing: run `make -C oracle ref` (needs /root/reference)")
    only = set(sys.argv[1:])
    path = os.path.join(HERE, "fullsize.json")
    out = json.load(open(path)) if os.path.exists(path) else []
    have = {(e["corpus"], e["codec"], e["chunk"], e["level"], e["size"]) for e in out}
    datas = {}
    for corpus, codec, chunk, level, size in WORKLOADS:
        if (corpus, codec, chunk, level, size) in have or (only and codec not in only):
            continue
        if (corpus, size) not in datas:
            datas = {(corpus, size): L.datagen(corpus, size, seed=SEED)}
        data = datas[(corpus, size)]
        packed, cs = O.compress_chunks(data, codec, chunk, level, use_ref=True, threads=8)
        e = {"corpus": corpus, "size": size, "seed": SEED, "codec": codec, "chunk": chunk, "level": level,
             "input_sha256": sha(data), "packed_sha256": sha(packed), "csizes_sha256": sha(cs.astype("<u8")),
             "packed_bytes": int(len(packed)), "ratio_pct": round(100 * len(packed) / size, 3)}
        print(e, flush=True)
        out.append(e)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
    shared(out, path, only)


if __name__ == "__main__":
    main()
