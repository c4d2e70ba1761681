"""tools/lz4split_ab.py -- lz4 -b64 compress (parse + emission + scan / pack): chunks split over the side
stream (lzh_debug_lz4_split 1) against both kernels on the caller's stream (0); HIP-event time of
DeviceCodec.compress, best of 8 alternating reps; packed bytes equal."""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch, lzbench_amd as L
split = L.lib().lzh_debug_lz4_split
split.restype = C.c_int
split.argtypes = [C.c_int]
for corpus, mib in (("text", 1024), ("text", 256), ("json", 1024)):
    n = mib << 20
    host = L.datagen(corpus, n, seed=12345)
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
    d_in[:n].copy_(torch.from_numpy(host))
    dc = L.DeviceCodec("lz4", n, 64 << 10)
    best = {0: 1e9, 1: 1e9}
    ref = None
    for r in range(8):
        for on in (1, 0):
            split(on)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            dc.compress(d_in)
            b.record()
            torch.cuda.synchronize()
            best[on] = min(best[on], a.elapsed_time(b))
            got = dc.packed[:dc.packed_total()].cpu()
            if ref is None:
                ref = got
            assert torch.equal(got, ref), (corpus, mib, on)
    split(1)
    print(f"lz4 {corpus} {mib} MiB compress: split {best[1]:.3f} ms, serial {best[0]:.3f} ms", flush=True)
