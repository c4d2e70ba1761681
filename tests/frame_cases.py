"""Shared helpers of the framed-format tests (LZ4 frame, nvcomp LZ4 container)."""
import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def golden():
    return json.load(open(os.path.join(HERE, "golden", "frames.json")))


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def key(c) -> str:
    return f"{c['codec']}-{c['corpus']}-{c['size']}-{c['chunk']}-{c['level']:#x}"


def corrupt(rng, s: bytes) -> bytes:
    """One random corruption of a frame: byte replacements, a bit flip in the header region,
    truncation, garbage appended, or a block word rewritten."""
    b = bytearray(s)
    kind = int(rng.integers(0, 5))
    if kind == 0:
        for _ in range(int(rng.integers(1, 4))):
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
    elif kind == 1:
        i = int(rng.integers(0, min(48, len(b))))
        b[i] ^= 1 << int(rng.integers(0, 8))
    elif kind == 2:
        b = b[: int(rng.integers(1, len(b)))]
    elif kind == 3:
        b += bytes(rng.integers(0, 256, int(rng.integers(1, 9)), dtype=np.uint8))
    else:
        i = int(rng.integers(0, max(1, len(b) - 4)))
        b[i:i + 4] = int(rng.integers(0, 1 << 32)).to_bytes(4, "little")
    return bytes(b)


def near_limit_blocks(rng, nblocks, bs=65536):
    """Blocks whose LZ4 size lands near the raw limit (bs - 1): random bytes with copies of earlier
    bytes spliced in at a per-block density, some copies reaching back into the previous block."""
    d = rng.integers(0, 256, nblocks * bs + int(rng.integers(0, 5000)), dtype=np.uint8)
    for b in range(nblocks):
        for _ in range(int(rng.integers(150, 330))):
            dst = b * bs + int(rng.integers(8, bs - 8))
            src = dst - int(rng.integers(4, 65535 if rng.random() < 0.2 else 4000))
            if src >= 0:
                ln = int(rng.integers(8, 17))
                d[dst:dst + ln] = d[src:src + ln].copy()
    return d
