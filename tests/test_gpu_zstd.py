"""GPU zstd decoder (LZH_CODEC_ZSTD, decode_hip.hip zstdd::) on frames written by the REFERENCE
zstd 1.5.2 with lzbench's zstd-row parameters (compressors.cpp:1745-1773): the committed golden
frames, fresh frames over corpora x chunk sizes x levels (raw, RLE and compressed blocks,
predefined / RLE / FSE / repeat tables, 1- and 4-stream Huffman literals, multi-block frames),
edge sizes, and corrupted frames (no fault; the reference's accept / reject verdict, and its bytes).
Parity is exact: the decoded bytes must equal the original input.  The decoder has two paths: the
split kernels (header / sequences one frame per lane / execution) and the one-wave-per-frame kernel
that takes the frames the split layout does not fit; `path` runs a test through each (the
lzh_debug_zstd_legacy hook forces the second).  Run with -m gpu."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import lzbench_amd as L
from test_zstd_golden import arrays, cases, corpus

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    return torch


# split: the four kernels (the literal kernel's sections per wave by frame count: 4 for these sizes; streams
# of 4096 symbols and more a wave each, lzh_zstd_hufpar_kernel); split8: the same with 8 sections a wave
# forced (lzh_debug_zstd_huf_sections); nopar: every stream one lane (lzh_debug_zstd_hufpar off) and every
# kernel on the caller's stream in order (lzh_debug_zstd_side off: by default the sequence kernel runs on a
# side stream beside the literal kernels; split and split8 differ there too: split plans the sequence kernel in
# two launches by sequence count, lzh_zstd_plan_kernel, split8 runs one -- lzh_debug_zstd_plan); legacy: the
# one-wave decoder
PATHS = ["split", "split8", "nopar", "legacy"]


def _legacy(on):
    f = L.lib().lzh_debug_zstd_legacy
    f.restype = C.c_int
    f.argtypes = [C.c_int]
    assert f(1 if on else 0) == 0


def _hufpar(on):
    f = L.lib().lzh_debug_zstd_hufpar
    f.restype = C.c_int
    f.argtypes = [C.c_int]
    assert f(1 if on else 0) == 0


def _side(on):
    f = L.lib().lzh_debug_zstd_side
    f.restype = C.c_int
    f.argtypes = [C.c_int]
    assert f(1 if on else 0) == 0


def _plan(on):
    f = L.lib().lzh_debug_zstd_plan
    f.restype = C.c_int
    f.argtypes = [C.c_int]
    assert f(1 if on else 0) == 0


def _huf_sections(hj):
    f = L.lib().lzh_debug_zstd_huf_sections
    f.restype = C.c_int
    f.argtypes = [C.c_int]
    assert f(hj) == 0


def gpu_decode(torch, packed, cs, n, chunk, path="split"):
    dc = L.DeviceCodec("zstd", n, chunk)
    d_packed = torch.zeros(len(packed) + 256, dtype=torch.uint8, device="cuda")
    if len(packed):
        d_packed[:len(packed)].copy_(torch.from_numpy(np.array(packed, dtype=np.uint8)))
    d_cs = torch.from_numpy(np.asarray(cs).astype(np.int32)).cuda()
    dc.out.fill_(0xA5)
    try:
        _legacy(path == "legacy")
        _huf_sections(8 if path == "split8" else 0)
        _hufpar(path != "nopar")
        _side(path != "nopar")
        _plan(path != "split8")
        dc.decompress(packed=d_packed, csizes=d_cs)
        torch.cuda.synchronize()
    finally:
        _legacy(False)
        _huf_sections(0)
        _hufpar(True)
        _side(True)
        _plan(True)
    return dc.status[:dc.k].cpu().numpy(), dc.out[:n].cpu().numpy()


def expected_sizes(n, chunk):
    k = (n + chunk - 1) // chunk
    return np.array([min(chunk, n - i * chunk) for i in range(k)])


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("case", cases(), ids=lambda c: c["name"])
def test_golden_frames(torch_cuda, case, path):
    A = arrays()
    data = corpus(case)
    st, out = gpu_decode(torch_cuda, A[case["name"] + "/packed"], A[case["name"] + "/csizes"], len(data), case["chunk"],
                         path)
    assert (st == expected_sizes(len(data), case["chunk"])).all(), st
    assert (out == data).all()


@pytest.mark.parametrize("level", [1, 2, 3, 5, 9, 19])
@pytest.mark.parametrize("chunk", [65536, 131072, 524288])
@pytest.mark.parametrize("kind", ["text", "json", "binary", "mixed"])
def test_reference_frames(torch_cuda, kind, chunk, level):
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    if level >= 9 and chunk != 131072:
        pytest.skip("slow CPU compression; one chunk size is enough")
    data = L.datagen(kind, 3 << 20 if level < 9 else 1 << 20, 23 + level)
    packed, cs = O.compress_chunks(data, "zstd", chunk, level)
    st, out = gpu_decode(torch_cuda, packed, cs, len(data), chunk)
    assert (st == expected_sizes(len(data), chunk)).all(), np.unique(st)
    assert (out == data).all()


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("n", [1, 5, 13, 255, 4096 + 3, 131072 - 1, 131072 + 1, 3 * 131072 + 77])
def test_edge_sizes(torch_cuda, n, path):
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    data = L.datagen("text", n, 7)
    packed, cs = O.compress_chunks(data, "zstd", 131072, 1)
    st, out = gpu_decode(torch_cuda, packed, cs, n, 131072, path)
    assert (st == expected_sizes(n, 131072)).all() and (out == data).all()


def _corrupt(rng, s: bytes) -> bytes:
    b = bytearray(s)
    kind = int(rng.integers(0, 4))
    if kind == 0:
        for _ in range(int(rng.integers(1, 4))):
            b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
    elif kind == 1:
        i = int(rng.integers(0, len(b)))
        b[i] ^= 1 << int(rng.integers(0, 8))
    elif kind == 2:
        b = b[: int(rng.integers(1, len(b)))]
    else:
        b += bytes(rng.integers(0, 256, int(rng.integers(1, 64))).astype(np.uint8))
    return bytes(b)


def _verdicts(torch, streams, chunk, path="split"):
    """GPU decode of every stream; the (index, gpu, reference) triples whose accept / reject verdicts
    differ (lzbench's length check: a frame is accepted when it decodes to exactly `chunk` bytes), and
    asserts the bytes of every frame both accept are the reference's."""
    blob = np.frombuffer(b"".join(streams), np.uint8)
    st, out = gpu_decode(torch, blob, [len(s) for s in streams], len(streams) * chunk, chunk, path)
    R = O.ref()
    mism = []
    for i, s in enumerate(streams):
        src = np.frombuffer(s, np.uint8).copy()
        dst = np.zeros(chunk + 64, np.uint8)
        r = R.ref_zstd_decompress(src.ctypes.data, len(s), dst.ctypes.data, chunk)
        if (st[i] == chunk) != (r == chunk):
            mism.append((i, int(st[i]), int(r)))
        elif r == chunk:
            assert (out[i * chunk:(i + 1) * chunk] == dst[:chunk]).all(), f"stream {i}: bytes differ"
    return mism, int((st == chunk).sum())


def _plain_frames(kind, chunk, seed):
    data = L.datagen(kind, 8 * chunk, seed)
    packed, cs = O.compress_chunks(data, "zstd", chunk, 1)
    offs = np.concatenate([[0], np.cumsum(cs)]).astype(np.int64)
    return [packed[offs[i]:offs[i + 1]].tobytes() for i in range(len(cs)) if cs[i] != chunk]


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("corpus_kind", ["text", "json", "mixed"])
def test_corrupt_frames(torch_cuda, corpus_kind, path):
    """1024 randomly corrupted plain (unchecksummed) frames per corpus: the decoder never faults and
    its accept / reject verdict equals ZSTD_decompressDCtx's frame for frame (including the literal
    sections the reference decodes with the double-symbol Huffman decoder: HUF_selectDecoder,
    huf_decompress.c:1593-1615), with the same bytes when both accept."""
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    chunk = 32768
    rng = np.random.default_rng(5 + len(corpus_kind))
    valid = _plain_frames(corpus_kind, chunk, 31)
    streams = []
    while len(streams) < 1024:
        s = _corrupt(rng, valid[int(rng.integers(0, len(valid)))])
        if 0 < len(s) != chunk:
            streams.append(s)
    mism, accepted = _verdicts(torch_cuda, streams, chunk, path)
    assert not mism, mism[:10]
    assert accepted > 0


def _huf_stream_spans(frame: bytes):
    """Byte ranges [a, b) of the Huffman literal streams of every compressed block of a frame
    (RFC 8878 3.1.1.3.1; 4-stream sections: the jump table is included as its own 6-byte span)."""
    fhd = frame[4]
    p = 5 + (0 if (fhd >> 5) & 1 else 1)
    p += (0, 1, 2, 4)[fhd & 3]
    fcsf = fhd >> 6
    p += (1 if (fhd >> 5) & 1 else 0, 2, 4, 8)[fcsf]
    spans = []
    while p + 3 <= len(frame):
        bh = frame[p] | frame[p + 1] << 8 | frame[p + 2] << 16
        p += 3
        last, btype, bsz = bh & 1, (bh >> 1) & 3, bh >> 3
        if btype == 2 and (frame[p] & 3) >= 2:
            b0, sf = frame[p], (frame[p] >> 2) & 3
            hsz = 3 if sf <= 1 else (4 if sf == 2 else 5)
            bits = 10 if sf <= 1 else (14 if sf == 2 else 18)
            h = int.from_bytes(frame[p:p + hsz], "little")
            cs = (h >> (4 + bits)) & ((1 << bits) - 1)
            q = p + hsz
            if b0 & 3 == 2:
                hb = frame[q]
                q += 1 + (hb if hb < 128 else (hb - 127 + 1) // 2)
            end = p + hsz + cs
            if sf == 0:
                spans.append((q, end))
            else:
                z1, z2, z3 = (int.from_bytes(frame[q + 2 * j:q + 2 * j + 2], "little") for j in range(3))
                spans.append((q, q + 6))
                a = q + 6
                for z in (z1, z2, z3):
                    spans.append((a, a + z))
                    a += z
                spans.append((a, end))
        p += bsz if btype != 1 else 1
        if last:
            break
    return [(a, b) for a, b in spans if 0 <= a < b <= len(frame)]


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("corpus_kind,chunk", [("text", 32768), ("json", 65536), ("mixed", 131072)])
def test_corrupt_huffman_streams(torch_cuda, corpus_kind, chunk, path):
    """1024 frames per case corrupted inside the Huffman literal streams -- their first and last bytes
    (where the double-symbol decoder's last-symbol step and the 4-stream loop's bounds decide), the
    jump table, anywhere in a stream: verdict and bytes equal ZSTD_decompressDCtx's."""
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    rng = np.random.default_rng(91 + chunk)
    valid = [(f, _huf_stream_spans(f)) for f in _plain_frames(corpus_kind, chunk, 57)]
    valid = [(f, sp) for f, sp in valid if sp]
    assert valid
    streams = []
    while len(streams) < 1024:
        f, sp = valid[int(rng.integers(0, len(valid)))]
        a, b = sp[int(rng.integers(0, len(sp)))]
        buf = bytearray(f)
        where = int(rng.integers(0, 3))
        i = (a + int(rng.integers(0, min(3, b - a)))) if where == 0 else \
            (b - 1 - int(rng.integers(0, min(3, b - a)))) if where == 1 else int(rng.integers(a, b))
        if rng.integers(0, 2):
            buf[i] ^= 1 << int(rng.integers(0, 8))
        else:
            buf[i] = int(rng.integers(0, 256))
        s = bytes(buf)
        if s != f:
            streams.append(s)
    mism, accepted = _verdicts(torch_cuda, streams, chunk, path)
    assert not mism, mism[:10]
    assert accepted > 0


def _ref_checksum_frames(data, chunk, level):
    R = O.ref()
    frames = []
    for i in range(0, len(data), chunk):
        part = np.ascontiguousarray(data[i:i + chunk])
        out = np.zeros(len(part) + len(part) // 8 + 1024, np.uint8)
        r = R.ref_zstd_compress_checksum(part.ctypes.data, len(part), out.ctypes.data, len(out), level)
        assert r > 0
        frames.append(out[:r].tobytes())
    return frames


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("kind,chunk,level", [("text", 131072, 1), ("json", 65536, 1), ("mixed", 1 << 20, 1),
                                              ("random", 131072, 1), ("binary", 100000, -3)])
def test_checksummed_frames(torch_cuda, kind, chunk, level, path):
    """Frames with the XXH64 content checksum (fParams.checksumFlag): decoded and verified."""
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    torch = torch_cuda
    n = 3 * chunk + 777
    data = L.datagen(kind, n, seed=13)
    frames = _ref_checksum_frames(data, chunk, level)
    frames = [f if len(f) != min(chunk, n - i * chunk) else None for i, f in enumerate(frames)]
    if any(f is None for f in frames):
        pytest.skip("a frame came out exactly chunk-sized (would read as stored raw)")
    st, out = gpu_decode(torch, np.frombuffer(b"".join(frames), np.uint8), [len(f) for f in frames], n, chunk, path)
    assert (st == expected_sizes(n, chunk)).all() and (out == data).all()
    # a wrong checksum is rejected, as by the reference
    bad = [bytearray(f) for f in frames]
    for b in bad:
        b[-1 - (len(b) % 4)] ^= 0x10
    st2, _ = gpu_decode(torch, np.frombuffer(b"".join(bytes(b) for b in bad), np.uint8), [len(b) for b in bad], n, chunk,
                        path)
    R = O.ref()
    for i, b in enumerate(bad):
        src = np.frombuffer(bytes(b), np.uint8).copy()
        dst = np.zeros(chunk + 64, np.uint8)
        r = R.ref_zstd_decompress(src.ctypes.data, len(b), dst.ctypes.data, chunk)
        assert (st2[i] >= 0) == (r >= 0), (i, st2[i], r)


@pytest.mark.parametrize("path", PATHS)
@pytest.mark.parametrize("corpus_kind", ["text", "json"])
def test_corrupt_checksummed_frames_verdicts(torch_cuda, corpus_kind, path):
    """Corrupted checksummed frames: with the content checksum on, the GPU decoder's verdict equals
    the reference's (ZSTD_decompressDCtx) frame for frame, and accepted frames decode identically."""
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    torch = torch_cuda
    chunk = 32768
    rng = np.random.default_rng(17 + len(corpus_kind))
    data = L.datagen(corpus_kind, 8 * chunk, 41)
    valid = _ref_checksum_frames(data, chunk, 1)
    streams = []
    while len(streams) < 1024:
        s = _corrupt(rng, valid[int(rng.integers(0, len(valid)))])
        if 0 < len(s) != chunk:
            streams.append(s)
    blob = np.frombuffer(b"".join(streams), np.uint8)
    st, out = gpu_decode(torch, blob, [len(s) for s in streams], len(streams) * chunk, chunk, path)
    R = O.ref()
    mism = []
    for i, s in enumerate(streams):
        src = np.frombuffer(s, np.uint8).copy()
        dst = np.zeros(chunk + 64, np.uint8)
        r = R.ref_zstd_decompress(src.ctypes.data, len(s), dst.ctypes.data, chunk)
        # (a frame of another content size is not this chunk's: lzbench's length check fails it)
        if (st[i] == chunk) != (r == chunk):
            mism.append((i, int(st[i]), int(r)))
        elif r >= 0:
            assert (out[i * chunk:(i + 1) * chunk] == dst[:chunk]).all(), f"stream {i}: bytes differ"
    assert not mism, mism[:10]


@pytest.mark.parametrize("corpus_kind,chunk", [("text", 32768), ("mixed", 131072)])
def test_split_and_legacy_statuses_equal(torch_cuda, corpus_kind, chunk):
    """The two paths return the same status (size or error code) and bytes for every frame of a
    corrupted set, frame for frame."""
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    rng = np.random.default_rng(303 + chunk)
    valid = _plain_frames(corpus_kind, chunk, 77)
    streams = []
    while len(streams) < 512:
        s = _corrupt(rng, valid[int(rng.integers(0, len(valid)))])
        if 0 < len(s) != chunk:
            streams.append(s)
    blob = np.frombuffer(b"".join(streams), np.uint8)
    cs = [len(s) for s in streams]
    st1, out1 = gpu_decode(torch_cuda, blob, cs, len(streams) * chunk, chunk, "split")
    st2, out2 = gpu_decode(torch_cuda, blob, cs, len(streams) * chunk, chunk, "legacy")
    assert (st1 == st2).all(), np.nonzero(st1 != st2)[0][:10]
    for i in np.nonzero(st1 == chunk)[0]:
        assert (out1[i * chunk:(i + 1) * chunk] == out2[i * chunk:(i + 1) * chunk]).all(), i
    st3, out3 = gpu_decode(torch_cuda, blob, cs, len(streams) * chunk, chunk, "split8")
    assert (st3 == st2).all(), np.nonzero(st3 != st2)[0][:10]
    for i in np.nonzero(st3 == chunk)[0]:
        assert (out3[i * chunk:(i + 1) * chunk] == out2[i * chunk:(i + 1) * chunk]).all(), i


def _raw_block_frame(data: bytes, block: int) -> bytes:
    """A single-segment frame of raw blocks of `block` bytes (RFC 8878 3.1.1.2): more blocks than the
    split layout holds for its chunk size, so the frame goes to the one-wave decoder."""
    n = len(data)
    hdr = bytearray(b"\x28\xb5\x2f\xfd")
    hdr.append(0x20 | (2 << 6))          # single segment, 4-byte content size
    hdr += n.to_bytes(4, "little")
    out = bytearray(hdr)
    for i in range(0, n, block):
        part = data[i:i + block]
        last = 1 if i + block >= n else 0
        bh = last | (0 << 1) | (len(part) << 3)
        out += bh.to_bytes(3, "little") + part
    return bytes(out)


@pytest.mark.parametrize("path", PATHS)
def test_many_block_frames_take_the_one_wave_decoder(torch_cuda, path):
    chunk = 131072
    data = L.datagen("text", 4 * chunk, 5)
    frames = [_raw_block_frame(data[i:i + chunk].tobytes(), 1000) for i in range(0, len(data), chunk)]
    st, out = gpu_decode(torch_cuda, np.frombuffer(b"".join(frames), np.uint8), [len(f) for f in frames], len(data), chunk,
                         path)
    assert (st == chunk).all(), st
    assert (out == data).all()


def test_long_literal_streams_wave_parallel(torch_cuda):
    """mixed -b128: a third of its frames are whole-block literals (4 streams of 32 K symbols), decoded a wave
    a stream; the bytes and statuses equal the per-lane decode's and the input"""
    torch = torch_cuda
    n, chunk = 24 << 20, 131072
    data = L.datagen("mixed", n, seed=12345)
    packed, cs = L.compress_chunks(data, "zstd", chunk, 1)
    st, out = gpu_decode(torch, packed, cs, n, chunk, "split")
    st0, out0 = gpu_decode(torch, packed, cs, n, chunk, "nopar")
    assert (st == expected_sizes(n, chunk)).all() and (st == st0).all()
    assert (out == data).all() and (out0 == data).all()


def _rle_seq_frame(nseq: int, n: int = 131072) -> bytes:
    """A single-segment frame of one compressed block (RFC 8878 3.1.1.3): nseq raw literals and nseq sequences
    with RLE-coded LL / OF / ML codes 1 / 0 / 52 -- literal length 1, repcode 1 (offset 1), match length
    65539 + 16 extra bits, all 0xFFFC: 131071 -- so every sequence adds 2^17 output bytes.  nseq = 1 is a valid
    frame of exactly n = 2^17 bytes; nseq = 32769 sums the sequences to 2^32 + 2^17, which a 32-bit output
    position wraps to exactly n (the reference rejects it at its second sequence, ZSTD_execSequence)."""
    lit = bytes([0x41]) * nseq
    if nseq < 32:
        lh = bytes([nseq << 3])                                   # raw, 5-bit size
    else:
        lh = bytes([0x0C | ((nseq & 15) << 4), (nseq >> 4) & 0xFF, nseq >> 12])   # raw, 20-bit size
    if nseq < 128:
        sh = bytes([nseq])
    elif nseq < 0x7F00:
        sh = bytes([128 + (nseq >> 8), nseq & 0xFF])
    else:
        sh = bytes([255]) + (nseq - 0x7F00).to_bytes(2, "little")
    sh += bytes([(1 << 6) | (1 << 4) | (1 << 2), 1, 0, 52])     # LL / OF / ML RLE; their codes
    # the bitstream, read backwards: per sequence 0 offset bits, 16 ML bits, 0 LL bits (RLE states: 0 bits)
    bits = (0xFFFC).to_bytes(2, "little") * nseq + b"\x01"     # (the end marker)
    body = lh + lit + sh + bits
    fh = b"\x28\xb5\x2f\xfd" + bytes([0x20 | (2 << 6)]) + n.to_bytes(4, "little")
    return fh + (1 | (2 << 1) | (len(body) << 3)).to_bytes(3, "little") + body


@pytest.mark.parametrize("path", PATHS)
def test_sequences_past_2_31_output_bytes(torch_cuda, path):
    """(round-5 advisor) sequences whose lengths sum past 2^31 -- a 32-bit output position wraps back into
    range -- get the reference's verdict on every path; the one-sequence frame of the same layout decodes exact"""
    chunk = 131072
    R = O.ref() if O.have_ref() else None
    frames = [_rle_seq_frame(1), _rle_seq_frame(32769)]
    expect = np.frombuffer(b"\x41" * chunk, np.uint8)
    if R is not None:
        for f, want in zip(frames, (chunk, None)):
            src = np.frombuffer(f, np.uint8).copy()
            dst = np.zeros(chunk + 64, np.uint8)
            r = R.ref_zstd_decompress(src.ctypes.data, len(f), dst.ctypes.data, chunk)
            assert (r == chunk) == (want == chunk), r
            if want == chunk:
                assert (dst[:chunk] == expect).all()
    st, out = gpu_decode(torch_cuda, np.frombuffer(b"".join(frames), np.uint8), [len(f) for f in frames], 2 * chunk,
                         chunk, path)
    assert st[0] == chunk and (out[:chunk] == expect).all(), st
    assert st[1] < 0, st
