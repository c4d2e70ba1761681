"""Snappy chunks of more than one 64 KiB fragment decode a fragment per wave (decode_hip.hip,
lzh_snappy_split_kernel): a tag walk finds the tag that starts every 64 KiB of output, the fragments
decode as headerless streams of exactly their size, and a chunk that does not split cleanly, or any
fragment of which fails, decodes whole through the serial decoder.

Checks:
* round trips at several chunk sizes, with the split path's chunk counter (lzh_debug_snappy_split_done)
  showing it ran where it should: by default for chunks of 8..64 fragments (512 KiB .. 4 MiB), with the
  test mode from 2 fragments;
* hand-built VALID streams the reference compressor never writes -- a literal across a fragment
  start, a copy reaching into the previous fragment -- decode to the right bytes through the
  fallback, while a stream that splits cleanly is decoded by fragments;
* corrupted -b256 streams: the same verdicts and bytes with the split on and off, and the reference
  decoder's verdicts (snappy::RawUncompress from oracle/_ref).
Run with -m gpu."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import lzbench_amd as L

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    return torch


def _split(mode: int):
    """0: every chunk whole; 1: the default (chunks of 8..64 fragments); 2: chunks of 2..64 fragments"""
    f = L.lib().lzh_debug_snappy_split
    f.restype = C.c_int
    f.argtypes = [C.c_int]
    assert f(mode) == 0


def _done(reset: bool = False) -> int:
    f = L.lib().lzh_debug_snappy_split_done
    f.restype = C.c_longlong
    f.argtypes = [C.c_int]
    v = f(1 if reset else 0)
    assert v >= 0
    return v


def _decode(torch, streams, chunk, n):
    """decode the chunk streams (chunk-sized outputs, the last n - (k-1) chunk) -> (statuses, output)"""
    blob = b"".join(streams)
    k = len(streams)
    d_packed = torch.zeros(len(blob) + 256, dtype=torch.uint8, device="cuda")
    d_packed[: len(blob)].copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    d_cs = torch.tensor([len(s) for s in streams], dtype=torch.int32, device="cuda")
    dc = L.DeviceCodec("snappy", n, chunk)
    dc.out.zero_()
    dc.decompress(packed=d_packed, csizes=d_cs)
    torch.cuda.synchronize()
    return dc.status[:k].cpu().numpy(), dc.out[:n].cpu().numpy()


# ---- a minimal snappy writer for hand-built streams (snappy format: varint length, then tags)
def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 128:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


class _Stream:
    def __init__(self):
        self.tags = bytearray()
        self.out = bytearray()

    def lit(self, b: bytes):
        n = len(b) - 1
        if n < 60:
            self.tags += bytes([n << 2])
        elif n < 256:
            self.tags += bytes([60 << 2, n])
        elif n < 65536:
            self.tags += bytes([61 << 2]) + n.to_bytes(2, "little")
        else:
            self.tags += bytes([62 << 2]) + n.to_bytes(3, "little")
        self.tags += b
        self.out += b

    def copy(self, off: int, ln: int):   # COPY_2, 1 <= ln <= 64
        assert 1 <= ln <= 64 and 0 < off <= len(self.out)
        self.tags += bytes([((ln - 1) << 2) | 2]) + off.to_bytes(2, "little")
        for _ in range(ln):
            self.out.append(self.out[-off])

    def bytes(self) -> bytes:
        return _varint(len(self.out)) + bytes(self.tags)


def _fill(s: _Stream, rng, upto: int, copies: bool):
    """random literals (and in-range copies) until the output is exactly `upto` bytes"""
    while len(s.out) < upto:
        room = upto - len(s.out)
        if copies and len(s.out) >= 64 and room >= 8 and rng.random() < 0.5:
            s.copy(int(rng.integers(1, min(len(s.out) % 65536 or 65536, 4096) + 1)), int(min(room, rng.integers(4, 65))))
        else:
            s.lit(rng.integers(0, 256, int(min(room, rng.integers(1, 300)))).astype(np.uint8).tobytes())


@pytest.mark.parametrize("mode,chunk", [(1, 131072), (1, 262144), (1, 1 << 20), (1, 4 << 20), (1, 5 << 20),
                                        (2, 131072), (2, 262144), (2, 100000), (2, 1 << 20)])
@pytest.mark.parametrize("corpus", ["mixed", "text"])
def test_split_round_trip(torch_cuda, mode, chunk, corpus):
    torch = torch_cuda
    n = 24 * (1 << 20) + 777                   # ragged last chunk
    host = L.datagen(corpus, n, seed=606)
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
    d_in[:n].copy_(torch.from_numpy(host))
    try:
        _split(mode)
        dc = L.DeviceCodec("snappy", n, chunk)   # (temp sized under the mode)
        dc.compress(d_in)
        _done(reset=True)
        dc.out.zero_()
        dc.decompress()
        torch.cuda.synchronize()
        split = _done()
    finally:
        _split(1)
    st = dc.status[: dc.k].cpu().numpy()
    parts = np.minimum(chunk, n - np.arange(dc.k, dtype=np.int64) * chunk)
    assert (st == parts).all(), f"statuses {st[st != parts][:4]}"
    assert torch.equal(dc.out[:n], d_in[:n])
    frags = -(-chunk // 65536)
    if frags > 64 or (mode == 1 and frags < 8):
        assert split == 0
    else:   # every chunk of more than one fragment that was not stored raw
        stored = int((dc.csizes[: dc.k].cpu().numpy() == parts).sum())
        multi = int((parts > 65536).sum())
        assert split == multi - stored, (split, multi, stored)


def test_unsplittable_streams_fall_back(torch_cuda):
    torch = torch_cuda
    rng = np.random.default_rng(7)
    chunk = 131072
    streams, outs = [], []
    # a literal across the fragment start
    s = _Stream()
    _fill(s, rng, 65500, True)
    s.lit(rng.integers(0, 256, 100).astype(np.uint8).tobytes())
    _fill(s, rng, chunk, True)
    streams.append(s.bytes()); outs.append(bytes(s.out))
    # a copy from fragment 1 into fragment 0 (valid snappy: the offset is inside the chunk)
    s = _Stream()
    _fill(s, rng, 65536, True)
    s.copy(1000, 64)
    _fill(s, rng, chunk, True)
    streams.append(s.bytes()); outs.append(bytes(s.out))
    # clean: every fragment's tags start at its first byte, copies inside it
    s = _Stream()
    _fill(s, rng, 65536, True)
    s.lit(rng.integers(0, 256, 70).astype(np.uint8).tobytes())
    _fill(s, rng, chunk, True)
    streams.append(s.bytes()); outs.append(bytes(s.out))
    n = chunk * len(streams)
    try:
        _split(2)   # (chunks of two fragments)
        _done(reset=True)
        st, out = _decode(torch, streams, chunk, n)
        split = _done()
    finally:
        _split(1)
    assert (st == chunk).all(), st
    for i, o in enumerate(outs):
        assert out[i * chunk:(i + 1) * chunk].tobytes() == o, f"stream {i}"
    # the clean stream only (its copies are drawn with offsets below the output position mod 64 KiB, so
    # none reaches into fragment 0); the other two fall back
    assert split == 1


def test_corrupt_split_streams_verdicts(torch_cuda):
    """256 corrupted -b256 streams: verdicts and bytes equal with the split on and off, and the reference
    decoder's verdicts"""
    import test_gpu_fuzz as F
    torch = torch_cuda
    cap = 262144
    rng = np.random.default_rng(4242)
    data = L.datagen("text", 8 * cap, seed=9)
    packed, cs = L.compress_chunks(data, "snappy", cap)
    offs = np.concatenate([[0], np.cumsum(cs)]).astype(np.int64)
    valid = [packed[offs[i]:offs[i + 1]].tobytes() for i in range(len(cs))]
    streams = []
    while len(streams) < 256:
        s = F._corrupt(rng, valid[int(rng.integers(0, len(valid)))])
        if 0 < len(s) != cap:
            streams.append(s)
    n = len(streams) * cap
    try:
        _split(2)
        st_on, out_on = _decode(torch, streams, cap, n)
        _split(0)
        st_off, out_off = _decode(torch, streams, cap, n)
    finally:
        _split(1)
    assert (st_on == st_off).all()
    for i in range(len(streams)):
        if st_on[i] >= 0:
            assert out_on[i * cap: i * cap + st_on[i]].tobytes() == out_off[i * cap: i * cap + st_on[i]].tobytes()
    if O.have_ref():
        R = O.ref()
        for i, s in enumerate(streams):
            ulen = F._varint(s)
            ok = False
            if ulen is not None and ulen <= cap:
                src = np.frombuffer(s, np.uint8).copy()
                dst = np.zeros(ulen + 64, np.uint8)
                ok = bool(R.ref_snappy_uncompress(src.ctypes.data, len(s), dst.ctypes.data))
            assert (st_on[i] >= 0) == ok, f"stream {i}: gpu {st_on[i]} reference {ok}"
            if ok:
                assert st_on[i] == ulen and out_on[i * cap: i * cap + ulen].tobytes() == dst[:ulen].tobytes()


def test_split_through_the_batch_rows(torch_cuda):
    """lzbench's chunk loop (lzbench_hip_decompress_batch, sub-batches with their own temp) at -b1024 takes
    the split path too, against the reference digest of the same stream"""
    n = 40 * (1 << 20) + 12345
    chunk = 1 << 20
    data = L.datagen("mixed", n, seed=77)
    packed, cs = L.compress_chunks(data, "snappy", chunk)
    if O.have_ref():
        rp, rcs = O.compress_chunks(data, "snappy", chunk, use_ref=True)
        assert (cs == rcs).all() and len(packed) == len(rp) and (packed == rp).all()
    _done(reset=True)
    out = L.decompress_chunks(packed, cs, n, "snappy", chunk)
    assert _done() > 0
    assert (out[:n] == data).all()
