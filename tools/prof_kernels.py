"""tools/prof_kernels.py -- run the codec kernels alone (for rocprofv3 --pmc / --kernel-trace).
usage: python tools/prof_kernels.py [--codec lz4] [--mib 256] [--corpus text] [--reps 2] [--v1]"""
import argparse, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
ap = argparse.ArgumentParser()
ap.add_argument("--codec", default="lz4")
ap.add_argument("--mib", type=int, default=256)
ap.add_argument("--chunk-kib", type=int, default=64)
ap.add_argument("--corpus", default="text")
ap.add_argument("--reps", type=int, default=2)
ap.add_argument("--decompress", action="store_true")
ap.add_argument("--level", type=int, default=0)
ap.add_argument("--zstd-legacy", action="store_true", help="zstd: the one-wave-per-frame decoder only")
a = ap.parse_args()
import torch
import lzbench_amd as L
n = a.mib << 20
host = L.datagen(a.corpus, n, seed=12345)
d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda")
d_in[:n].copy_(torch.from_numpy(host))
dc = L.DeviceCodec(a.codec, n, a.chunk_kib << 10, level=a.level)
dc.compress(d_in)
torch.cuda.synchronize()
if a.zstd_legacy:
    L.lib().lzh_debug_zstd_legacy(1)
t = time.time()
for _ in range(a.reps):
    if a.decompress:
        dc.decompress()
    else:
        dc.compress_kernel_only(d_in)
torch.cuda.synchronize()
print(f"{a.codec}{a.level or ''} {'dec' if a.decompress else 'comp'} {a.mib} MiB: {(time.time()-t)/a.reps*1e3:.2f} ms/rep, ratio {dc.packed_total()/n:.4f}", flush=True)
