"""tools/zside_ab.py -- zstd-1 -b128 decode at config 5's shares: the sequence kernel on the side stream
(lzh_debug_zstd_side 1, default) against everything on the caller's stream (0); HIP-event time of
DeviceCodec.decompress (the launcher's kernels), best of 10 alternating reps, bytes checked."""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch, lzbench_amd as L
side = L.lib().lzh_debug_zstd_side
side.restype = C.c_int
side.argtypes = [C.c_int]
for mib in (512, 1024):
    n = mib << 20
    host = L.datagen("mixed", n, seed=12345)
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
    d_in[:n].copy_(torch.from_numpy(host))
    dc = L.DeviceCodec("zstd", n, 128 << 10, level=1)
    dc.compress(d_in)
    torch.cuda.synchronize()
    best = {0: 1e9, 1: 1e9}
    for r in range(10):
        for on in (1, 0):
            side(on)
            dc.out.zero_()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            dc.decompress()
            b.record()
            torch.cuda.synchronize()
            best[on] = min(best[on], a.elapsed_time(b))
            assert torch.equal(dc.out[:n], d_in[:n]), (mib, on)
    side(1)
    print(f"{mib} MiB decode: side {best[1]:.3f} ms, serial {best[0]:.3f} ms", flush=True)
