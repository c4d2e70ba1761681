#!/usr/bin/env python3
"""tests/golden/make_frame_golden.py -- digests of the REFERENCE framed-format chunk loops.

Run in the build container (needs oracle/_ref/libref.so: lz4 1.9.3 incl. lz4frame.c / lz4hc.c /
xxhash.c compiled from /root/reference by `make -C oracle ref`).  Inputs come from
lzbench_amd.datagen (deterministic), so only digests are stored:

  lz4f   one LZ4 frame per chunk: LZ4F_compressFrame with the listed params (bits 0-2
         blockSizeID, 0x10 block checksum, 0x20 content checksum, 0x40 content size, 0x80 linked
         blocks, bits 8-15 acceleration), lzbench's raw-store rule per chunk
  nvlz4  one nvcomp LZ4 container per chunk around reference LZ4_compress_default blocks of
         1 << (15 + level) bytes (the layout itself is a restatement: nvcomp cannot be built)

Writes frames.json: [{codec, corpus, size, seed, chunk, level, packed_sha256, csizes_sha256,
packed_bytes}] with csizes as little-endian u64.
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

MiB = 1 << 20
# (codec, corpus, size, chunk, level)
CASES = [
    ("lz4f", "text", 8 * MiB, 65536, 0),
    ("lz4f", "text", 8 * MiB + 777, 65536, 0x70),
    ("lz4f", "json", 4 * MiB, 131072, 0x10),
    ("lz4f", "mixed", 8 * MiB, 1 << 20, 5),
    ("lz4f", "mixed", 6 * MiB + 12345, 100 * 1024, 0x34),
    ("lz4f", "random", 2 * MiB, 65536, 0x30),
    ("lz4f", "binary", 4 * MiB, 262144, 6 | 0x40),
    ("lz4f", "text", 16 * MiB, 16 * MiB, 7 | 0x70),
    ("lz4f", "text", 4 * MiB, 65536, 0x300),
    ("lz4f", "json", 4 * MiB + 3, 200 * 1024, 4 | 0x1100),
    # linked blocks (0x80 = LZ4F_blockLinked, what LZ4F_compressFrame does with default preferences)
    ("lz4f", "text", 8 * MiB, 131072, 0x80),
    ("lz4f", "mixed", 8 * MiB, 1 << 20, 0x80),
    ("lz4f", "json", 6 * MiB + 12345, 1 << 20, 5 | 0x80 | 0x20),
    ("lz4f", "random", 4 * MiB, 262144, 0x80 | 0x10),
    ("lz4f", "binary", 4 * MiB, 262144, 0x80 | 0x300),
    ("lz4f", "mixed", 6 * MiB + 7, 300 * 1024, 0x80 | 0x40),
    ("nvlz4", "text", 8 * MiB, 65536, 0),
    ("nvlz4", "json", 8 * MiB + 99, 1 << 20, 1),
    ("nvlz4", "mixed", 8 * MiB, 4 << 20, 3),
    ("nvlz4", "random", 2 * MiB, 65536, 0),
    ("nvlz4", "binary", 6 * MiB + 5, 3 << 20, 5),
]
SEED = 4242


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    if not O.have_ref():
        sys.exit("oracle/_ref/libref.so missing: run `make -C oracle ref` (needs /root/reference)")
    out = []
    for codec, corpus, size, chunk, level in CASES:
        data = L.datagen(corpus, size, seed=SEED)
        packed, cs = O.compress_chunks(data, codec, chunk, level, use_ref=True)
        out.append(dict(codec=codec, corpus=corpus, size=size, seed=SEED, chunk=chunk, level=level,
                        packed_sha256=sha(packed), csizes_sha256=sha(cs.astype("<u8")), packed_bytes=int(len(packed))))
        print(codec, corpus, size, chunk, hex(level), len(packed), flush=True)
    json.dump(out, open(os.path.join(HERE, "frames.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
