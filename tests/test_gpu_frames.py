"""GPU framed formats through the C-ABI: LZ4 frames (LZ4F_compressFrame with
independent or linked blocks) and nvcomp LZ4 containers, one per chunk, against the REFERENCE digests of
tests/golden/frames.json and the reference build; decoding of reference frames and of corrupted
frames (verdicts against the CPU restatement, itself pinned to the reference LZ4F_decompress by
tests/test_frames.py).  Run with -m gpu."""
import ctypes as C

import numpy as np
import pytest

import frame_cases as F
import oracle_lib as O
import lzbench_amd as L

pytestmark = pytest.mark.gpu
NAME = {"lz4f": "lz4frame", "nvlz4": "nvcomp_lz4"}


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    return torch


@pytest.mark.parametrize("case", F.golden(), ids=F.key)
def test_frames_vs_reference_digests(torch_cuda, case):
    data = L.datagen(case["corpus"], case["size"], seed=case["seed"])
    name = NAME[case["codec"]]
    packed, cs = L.compress_chunks(data, name, case["chunk"], level=case["level"])
    assert len(packed) == case["packed_bytes"]
    assert F.sha(cs.astype("<u8")) == case["csizes_sha256"]
    assert F.sha(packed) == case["packed_sha256"]
    out = L.decompress_chunks(packed, cs, len(data), name, case["chunk"])
    assert (out == data).all()


@pytest.mark.parametrize("codec", ["lz4f", "nvlz4"])
@pytest.mark.parametrize("n,chunk", [(1, 65536), (12, 65536), (13, 64), (65535, 65536), (65537, 65536),
                                     (300001, 65536), (300001, 100000), (5 << 20, 1 << 22), (777777, 777777)])
def test_frames_edge_sizes_vs_restatement(torch_cuda, codec, n, chunk):
    levels = [0, 5, 0x74, 0x204, 0x80, 0x84, 0xF4, 0x380] if codec == "lz4f" else [0, 2, 5]
    for kind in ("text", "random"):
        data = L.datagen(kind, n, seed=n)
        for lvl in levels:
            exp, ecs = O.compress_chunks(data, codec, chunk, lvl)
            packed, cs = L.compress_chunks(data, NAME[codec], chunk, level=lvl)
            assert (cs == ecs).all() and len(packed) == len(exp) and (packed == exp).all(), (kind, hex(lvl))
            out = L.decompress_chunks(packed, cs, n, NAME[codec], chunk)
            assert (out == data).all()


def test_lz4frame_row_per_chunk_abi(torch_cuda):
    """The per-chunk row entry points (lzbench_hip_lz4frame_*), as lzbench's chunk loop calls them."""
    lib = L.lib()
    data = L.datagen("json", 200000, seed=3)
    for lvl, fn_c, fn_d, init, codec in ((4, "lzbench_hip_lz4frame_compress", "lzbench_hip_lz4frame_decompress",
                                          "lzbench_hip_lz4frame_init", "lz4f"),
                                         (2, "lzbench_hip_nvcomp_lz4_compress", "lzbench_hip_nvcomp_lz4_decompress",
                                          "lzbench_hip_nvcomp_lz4_init", "nvlz4")):
        wm = getattr(lib, init)(len(data), lvl, 1)
        assert wm
        try:
            out = np.zeros(len(data) * 2 + 65536, np.uint8)
            r = getattr(lib, fn_c)(data.ctypes.data, len(data), out.ctypes.data, len(out), lvl, 0, wm)
            exp, ecs = O.compress_chunks(data, codec, len(data), lvl)
            assert r == int(ecs[0]) and (out[:r] == exp).all()
            back = np.zeros(len(data) + 64, np.uint8)
            d = getattr(lib, fn_d)(out.ctypes.data, r, back.ctypes.data, len(data), lvl, 0, wm)
            assert d == len(data) and (back[:len(data)] == data).all()
        finally:
            lib.lzbench_hip_deinit(wm)


def test_device_resident_frames(torch_cuda):
    torch = torch_cuda
    n, chunk = (32 << 20) + 4321, 1 << 20
    data = L.datagen("mixed", n, seed=77)
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
    d_in[:n].copy_(torch.from_numpy(data))
    for name, codec, lvl in (("lz4frame", "lz4f", 0x70), ("lz4frame", "lz4f", 6), ("nvcomp_lz4", "nvlz4", 1)):
        dc = L.DeviceCodec(name, n, chunk, level=lvl)
        dc.compress(d_in)
        dc.decompress()
        torch.cuda.synchronize()
        total = dc.packed_total()
        exp, ecs = O.compress_chunks(data, codec, chunk, lvl)
        assert total == len(exp)
        assert (dc.csizes.cpu().numpy().astype(np.uint64) == ecs).all()
        assert (dc.packed[:total].cpu().numpy() == exp).all()
        assert (dc.status.cpu().numpy() == np.minimum(chunk, n - np.arange(dc.k) * chunk)).all()
        assert (dc.out[:n].cpu().numpy() == data).all()


@pytest.mark.parametrize("codec,params", [("lz4f", 0), ("lz4f", 0x70), ("lz4f", 0x15), ("lz4f", 0x80), ("lz4f", 0xB0),
                                          ("nvlz4", 0)])
def test_corrupt_frames_verdicts(torch_cuda, codec, params):
    torch = torch_cuda
    if codec == "lz4f" and not O.have_ref():
        pytest.skip("reference build not present")
    rng = np.random.default_rng(3 + params)
    part = 70000
    data = L.datagen("text", 8 * part, seed=21)
    packed, cs = O.compress_chunks(data, codec, part, params)
    offs = np.concatenate([[0], np.cumsum(cs)]).astype(np.int64)
    valid = [packed[offs[i]:offs[i + 1]].tobytes() for i in range(len(cs))]
    frames = []
    while len(frames) < 512:
        i = int(rng.integers(0, len(valid)))
        s = F.corrupt(rng, valid[i]) if len(frames) % 8 else valid[i]
        if 0 < len(s) != part:
            frames.append((i, s))
    blob = b"".join(s for _, s in frames)
    k = len(frames)
    d_packed = torch.zeros(len(blob) + 256, dtype=torch.uint8, device="cuda")
    d_packed[: len(blob)].copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    d_cs = torch.tensor([len(s) for _, s in frames], dtype=torch.int32, device="cuda")
    dc = L.DeviceCodec(NAME[codec], k * part, part)
    dc.decompress(packed=d_packed, csizes=d_cs)
    torch.cuda.synchronize()
    status = dc.status[:k].cpu().numpy()
    out = dc.out[: k * part].cpu().numpy()
    orc = O.oracle()
    fn = orc.oracle_lz4f_decompress if codec == "lz4f" else orc.oracle_nvlz4_decompress
    for j, (i, s) in enumerate(frames):
        src = np.frombuffer(s, np.uint8).copy()
        dst = np.zeros(part + 64, np.uint8)
        r = fn(src.ctypes.data, len(s), dst.ctypes.data, part)
        st = int(status[j])
        if r >= 0 and r != part:
            r = -1   # (a frame of another size is not this chunk's)
        assert (st >= 0) == (r >= 0), f"frame {j}: gpu {st} restatement {r}"
        if r >= 0:
            assert out[j * part:(j + 1) * part].tobytes() == dst[:part].tobytes()
        elif r == -2:
            assert st == -2


@pytest.mark.parametrize("params", [0x80, 0x90, 0x280])
def test_linked_frames_near_the_raw_limit(torch_cuda, params):
    """Linked frames (LZ4F's default) whose blocks barely do or do not fit size - 1 bytes: a failing
    block is stored raw and the next block starts from the table as the reference left it at the
    failing check (oracle/frame_oracle.c lz4f_linked_block, pinned to LZ4F_compressFrame by
    tests/test_frames.py), so every later block's bytes check the GPU's abort point and replay."""
    rng = np.random.default_rng(params)
    chunk = 5 * 65536
    data = np.concatenate([F.near_limit_blocks(rng, 5)[:chunk] for _ in range(12)])
    exp, ecs = O.compress_chunks(data, "lz4f", chunk, params)
    packed, cs = L.compress_chunks(data, "lz4frame", chunk, level=params)
    assert (cs == ecs).all() and len(packed) == len(exp) and (packed == exp).all()
    out = L.decompress_chunks(packed, cs, len(data), "lz4frame", chunk)
    assert (out == data).all()


def _with_dict_id(frame: bytes, flip_only: bool) -> bytes:
    """The frame with FLG's dictionary-id bit set.  flip_only: just the bit (the header checksum no
    longer matches); else a well-formed header: content size + dictionary id fields, checksum redone."""
    flg, bd = frame[4], frame[5]
    csz = (flg >> 3) & 1
    hl = 7 + 8 * csz
    if flip_only:
        b = bytearray(frame)
        b[4] ^= 1
        return bytes(b)
    body = frame[hl:]
    cs_field = frame[6:6 + 8] if csz else None
    hdr = bytearray([flg | 0x09, bd]) + (cs_field if csz else bytes(8)) + (0x1234567).to_bytes(4, "little")
    if not csz:
        return None
    h = np.frombuffer(bytes(hdr), np.uint8).copy()
    hc = (O.oracle().oracle_xxh32(h.ctypes.data, len(h), 0) >> 8) & 0xff
    return bytes(frame[:4]) + bytes(hdr) + bytes([hc]) + body


def test_dict_id_frames(torch_cuda):
    """A well-formed frame carrying a dictionary id (with content size: the 19-byte header, checksum
    over bytes 4..17) is refused as unsupported (-2) by the GPU and by the restatement alike; a frame
    whose dictionary-id bit alone was flipped fails LZ4F_decodeHeader's header checksum first (-1)."""
    torch = torch_cuda
    part = 70000
    data = L.datagen("text", 4 * part, seed=5)
    packed, cs = O.compress_chunks(data, "lz4f", part, 0x40)      # content size on
    offs = np.concatenate([[0], np.cumsum(cs)]).astype(np.int64)
    valid = [packed[offs[i]:offs[i + 1]].tobytes() for i in range(len(cs))]
    frames = [_with_dict_id(v, False) for v in valid] + [_with_dict_id(v, True) for v in valid]
    want = [-2] * len(valid) + [-1] * len(valid)
    orc = O.oracle()
    for s, w in zip(frames, want):
        src = np.frombuffer(s, np.uint8).copy()
        dst = np.zeros(part + 64, np.uint8)
        assert orc.oracle_lz4f_decompress(src.ctypes.data, len(s), dst.ctypes.data, part) == w
    blob = b"".join(frames)
    k = len(frames)
    d_packed = torch.zeros(len(blob) + 256, dtype=torch.uint8, device="cuda")
    d_packed[: len(blob)].copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    d_cs = torch.tensor([len(s) for s in frames], dtype=torch.int32, device="cuda")
    dc = L.DeviceCodec("lz4frame", k * part, part)
    dc.decompress(packed=d_packed, csizes=d_cs)
    torch.cuda.synchronize()
    assert dc.status[:k].cpu().numpy().tolist() == want
