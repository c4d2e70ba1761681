"""The LZ4 / snappy decoder comes in three output-window kernels (4, 8 and 16 KiB of LDS; the launch
picks the widest whose occupancy holds all its chunks, decode_hip.hip lzh_launch_decompress).  Every
window must decode the same streams to the same bytes and give the same verdicts: each test forces
one window through the lzh_debug_force_decode_window hook and checks the round trip (streams from
the GPU compressor, bit-exact with the reference elsewhere) and corrupted streams against the
reference decoders.  Run with -m gpu."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib as O
import lzbench_amd as L

pytestmark = pytest.mark.gpu
WINDOWS = [4096, 8192, 16384]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    torch.cuda.set_device(0)
    return torch


def _force(kw):
    f = L.lib().lzh_debug_force_decode_window
    f.restype = C.c_int
    f.argtypes = [C.c_int]
    assert f(kw) == 0


@pytest.mark.parametrize("window", WINDOWS)
@pytest.mark.parametrize("codec,corpus,chunk", [("lz4", "text", 65536), ("lz4", "binary", 262144),
                                                ("snappy", "mixed", 262144), ("snappy", "text", 65536),
                                                ("lz4", "json", 1 << 20)])
def test_window_round_trip(torch_cuda, window, codec, corpus, chunk):
    torch = torch_cuda
    n = 16 * (1 << 20) + 4321                   # ragged last chunk
    host = L.datagen(corpus, n, seed=2024)
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
    d_in[:n].copy_(torch.from_numpy(host))
    dc = L.DeviceCodec(codec, n, chunk)
    dc.compress(d_in)
    try:
        _force(window)
        dc.out.zero_()
        dc.decompress()
        torch.cuda.synchronize()
    finally:
        _force(0)
    st = dc.status[: dc.k].cpu().numpy()
    parts = np.minimum(chunk, n - np.arange(dc.k, dtype=np.int64) * chunk)
    assert (st == parts).all(), f"statuses {st[st != parts][:4]}"
    assert torch.equal(dc.out[:n], d_in[:n])


def test_window_hook_rejects_other_sizes():
    f = L.lib().lzh_debug_force_decode_window
    f.restype = C.c_int
    f.argtypes = [C.c_int]
    assert f(2048) == -1 and f(12345) == -1 and f(0) == 0


@pytest.mark.parametrize("window", WINDOWS)
@pytest.mark.parametrize("codec", ["lz4", "snappy"])
def test_window_corrupt_verdicts(torch_cuda, window, codec):
    """256 corrupted streams per window: verdict and bytes as the reference decoder's."""
    if not O.have_ref():
        pytest.skip("reference build (oracle/_ref) not present")
    import test_gpu_fuzz as F
    torch = torch_cuda
    rng = np.random.default_rng(31 + window + len(codec))
    data = L.datagen("text", 8 * F.CAP, seed=5)
    packed, cs = O.compress_chunks(data, codec, F.CAP)
    offs = np.concatenate([[0], np.cumsum(cs)]).astype(np.int64)
    valid = [packed[offs[i]:offs[i + 1]].tobytes() for i in range(len(cs))]
    streams = []
    while len(streams) < 256:
        s = F._corrupt(rng, valid[int(rng.integers(0, len(valid)))])
        if 0 < len(s) != F.CAP:
            streams.append(s)
    blob = b"".join(streams)
    k = len(streams)
    d_packed = torch.zeros(len(blob) + 256, dtype=torch.uint8, device="cuda")
    d_packed[: len(blob)].copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    d_cs = torch.tensor([len(s) for s in streams], dtype=torch.int32, device="cuda")
    dc = L.DeviceCodec(codec, k * F.CAP, F.CAP)
    try:
        _force(window)
        dc.decompress(packed=d_packed, csizes=d_cs)
        torch.cuda.synchronize()
    finally:
        _force(0)
    status = dc.status[:k].cpu().numpy()
    out = dc.out[: k * F.CAP].cpu().numpy()
    for i, s in enumerate(streams):
        r, ref_out = F._ref_verdict(codec, s)
        st = int(status[i])
        assert (st >= 0) == (r >= 0), f"stream {i}: gpu {st} reference {r}"
        if r >= 0:
            assert st == r
            assert out[i * F.CAP: i * F.CAP + r].tobytes() == ref_out
