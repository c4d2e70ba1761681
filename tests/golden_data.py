"""tests/golden_data.py -- loader for tests/golden (reference-generated vectors, see make_golden.py)."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN_DIR = os.path.join(HERE, "golden")
_npz = None
_manifest = None


def arrays():
    global _npz
    if _npz is None:
        with np.load(os.path.join(GOLDEN_DIR, "golden.npz"), allow_pickle=False) as z:
            _npz = {k: z[k] for k in z.files}
    return _npz


def manifest():
    global _manifest
    if _manifest is None:
        with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
            _manifest = json.load(f)
    return _manifest


def sha(*xs) -> str:
    h = hashlib.sha256()
    for a in xs:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def inp(name: str) -> np.ndarray:
    return arrays()[f"in/{name}"]


def block_cases(codec=None):
    return [c for c in manifest()["cases"] if c["kind"] == "block" and (codec is None or c["codec"] == codec)]


def chunk_cases():
    return [c for c in manifest()["cases"] if c["kind"] == "chunks"]


def check_block(case, got: bytes) -> bool:
    if len(got) != case["csize"]:
        return False
    if case["stored"]:
        return got == arrays()[case["key"]].tobytes()
    return sha(np.frombuffer(got, np.uint8)) == case["sha256"]
