"""Framed LZ4 formats on the CPU: the restatement (oracle/frame_oracle.c)
against the REFERENCE LZ4F build (lz4/lz4frame.c + lz4hc.c + xxhash.c compiled from /root/reference
into oracle/_ref) and against the reference digests in tests/golden/frames.json."""
import numpy as np
import pytest

import frame_cases as F
import oracle_lib as O
import lzbench_amd as L

SIZES = [0, 1, 5, 12, 13, 100, 4095, 4096, 65535, 65536, 65537, 65547, 200000, 262145, (1 << 20) + 17]
PARAMS = [0, 4, 5, 6, 7, 0x10, 0x20, 0x40, 0x74, 0x300, 0x1104, 0x77,
          0x80, 0x84, 0x85, 0xF4, 0x380, 0x1184]          # 0x80: linked blocks (the LZ4F default)


def _frame(fn, data, params, cap):
    out = np.zeros(cap, np.uint8)
    r = fn(data.ctypes.data, len(data), out.ctypes.data, params) if fn.__name__.startswith("oracle") else \
        fn(data.ctypes.data, len(data), out.ctypes.data, cap, params)
    return out[:r].tobytes() if r >= 0 else None


def test_xxh32_known_answers():
    orc = O.oracle()
    # XXH32 reference values (xxhash's published sanity checks, seed 0)
    assert orc.oracle_xxh32(None, 0, 0) == 0x02CC5D05
    d = np.frombuffer(b"abc", np.uint8).copy()
    assert orc.oracle_xxh32(d.ctypes.data, 3, 0) == 0x32D153FF


@pytest.mark.parametrize("kind", ["text", "json", "random", "binary"])
def test_lz4f_oracle_vs_reference(kind):
    if not O.have_ref():
        pytest.skip("reference build not present")
    R, orc = O.ref(), O.oracle()
    for n in SIZES:
        data = L.datagen(kind, n, seed=n + 3) if n else np.zeros(0, np.uint8)
        for p in PARAMS:
            cap = int(R.ref_lz4f_bound(n, p)) + 64
            a = _frame(R.ref_lz4f_compress, data, p, cap)
            b = _frame(orc.oracle_lz4f_compress, data, p, max(cap, int(orc.oracle_lz4f_bound(n, p))) + 64)
            assert a == b, (kind, n, hex(p))
            o = np.zeros(n + 64, np.uint8)
            ab = np.frombuffer(a, np.uint8).copy()
            assert orc.oracle_lz4f_decompress(ab.ctypes.data, len(a), o.ctypes.data, n + 64) == n
            assert (o[:n] == data).all()


def test_lz4f_raw_block_boundary():
    """Blocks that barely do or do not compress (LZ4F_makeBlock's dstCapacity = size - 1)."""
    if not O.have_ref():
        pytest.skip("reference build not present")
    R, orc = O.ref(), O.oracle()
    rng = np.random.default_rng(7)
    for t in range(400):
        n = int(rng.integers(1, 3000))
        d = rng.integers(0, 256, n, dtype=np.uint8)
        k = int(rng.integers(0, min(n, 64) + 1))
        d[:k] = d[0]
        a = _frame(R.ref_lz4f_compress, d, 0, n + 256)
        b = _frame(orc.oracle_lz4f_compress, d, 0, n + 256)
        assert a == b


def test_lz4f_linked_raw_decisions_vs_reference():
    """Linked frames whose blocks barely do or do not fit size - 1 bytes: a block that fails is stored
    raw and the parse stopped where the first limitedOutput check failed -- the next block starts from
    the table as it stood there (lz4.c:1024-1027, :1097-1121, :1207-1216), so the following blocks'
    bytes pin the abort point."""
    if not O.have_ref():
        pytest.skip("reference build not present")
    R, orc = O.ref(), O.oracle()
    rng = np.random.default_rng(17)
    raw = comp = 0
    for t in range(60):
        d = F.near_limit_blocks(rng, int(rng.integers(2, 6)))
        for p in (0x80, 0x90):
            cap = int(R.ref_lz4f_bound(len(d), p)) + 64
            a = _frame(R.ref_lz4f_compress, d, p, cap)
            b = _frame(orc.oracle_lz4f_compress, d, p, max(cap, int(orc.oracle_lz4f_bound(len(d), p))) + 64)
            assert a == b, (t, hex(p))
            o = np.zeros(len(d) + 64, np.uint8)
            ab = np.frombuffer(a, np.uint8).copy()
            assert orc.oracle_lz4f_decompress(ab.ctypes.data, len(a), o.ctypes.data, len(d) + 64) == len(d)
            assert (o[:len(d)] == d).all()
            # count raw / compressed blocks (both must occur for the test to mean something)
            ip = 7
            while True:
                w = int.from_bytes(a[ip:ip + 4], "little")
                ip += 4
                if w == 0:
                    break
                raw += w >> 31
                comp += 1 - (w >> 31)
                ip += (w & 0x7fffffff) + (4 if p & 0x10 else 0)
    assert raw > 20 and comp > 20, (raw, comp)


def test_nvlz4_oracle_vs_reference():
    if not O.have_ref():
        pytest.skip("reference build not present")
    for kind in ("text", "random", "mixed"):
        data = L.datagen(kind, 3 * 65536 + 999, seed=5)
        for lvl in range(6):
            a, ca = O.compress_chunks(data, "nvlz4", 150000, lvl, use_ref=True)
            b, cb = O.compress_chunks(data, "nvlz4", 150000, lvl)
            assert (ca == cb).all() and (a == b).all()
            r, out = O.decompress_chunks(b, cb, len(data), "nvlz4", 150000)
            assert r == len(data) and (out == data).all()


@pytest.mark.parametrize("case", F.golden(), ids=F.key)
def test_oracle_reproduces_reference_digests(case):
    data = L.datagen(case["corpus"], case["size"], seed=case["seed"])
    packed, cs = O.compress_chunks(data, case["codec"], case["chunk"], case["level"])
    assert len(packed) == case["packed_bytes"]
    assert F.sha(packed) == case["packed_sha256"] and F.sha(cs.astype("<u8")) == case["csizes_sha256"]


def test_lz4f_decode_verdicts_vs_reference():
    """Corrupted frames: the restated LZ4F_decompress accepts exactly what the reference accepts."""
    if not O.have_ref():
        pytest.skip("reference build not present")
    R, orc = O.ref(), O.oracle()
    rng = np.random.default_rng(11)
    n = 70000
    data = L.datagen("text", n, seed=9)
    checked = 0
    for t in range(900):
        p = int(rng.choice([0, 0x10, 0x20, 0x40, 0x70, 5, 0x80, 0xB0]))
        good = _frame(R.ref_lz4f_compress, data, p, int(R.ref_lz4f_bound(n, p)) + 64)
        bad = np.frombuffer(F.corrupt(rng, good), np.uint8).copy()
        o1, o2 = np.zeros(n + 64, np.uint8), np.zeros(n + 64, np.uint8)
        x = R.ref_lz4f_decompress(bad.ctypes.data, len(bad), o1.ctypes.data, n)
        y = orc.oracle_lz4f_decompress(bad.ctypes.data, len(bad), o2.ctypes.data, n)
        if y == -2:
            continue
        checked += 1
        assert (x >= 0) == (y >= 0), (t, x, y)
        if x >= 0:
            assert x == y and (o1[:x] == o2[:y]).all()
    assert checked > 800
