"""Run the GPU zstd decoder on reference frames (MiB of a corpus, -b chunk, level) for profilers."""
import argparse, os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import torch
import lzbench_amd as L, oracle_lib as O
ap = argparse.ArgumentParser()
ap.add_argument("--mib", type=int, default=256); ap.add_argument("--chunk", type=int, default=131072)
ap.add_argument("--level", type=int, default=1); ap.add_argument("--corpus", default="text"); ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()
data = L.datagen(a.corpus, a.mib << 20, 3)
packed, cs = O.compress_chunks(data, "zstd", a.chunk, a.level, threads=16)
n = len(data)
dc = L.DeviceCodec("zstd", n, a.chunk)
d_packed = torch.zeros(len(packed) + 256, dtype=torch.uint8, device="cuda")
d_packed[:len(packed)].copy_(torch.from_numpy(packed))
d_cs = torch.from_numpy(cs.astype(np.int32)).cuda()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(a.reps):
    s.record(); dc.decompress(packed=d_packed, csizes=d_cs); e.record(); torch.cuda.synchronize(); ts.append(s.elapsed_time(e))
ok = bool((dc.out[:n].cpu().numpy() == data).all())
print(f"zstd decode {a.corpus} {a.mib} MiB -b{a.chunk >> 10} l{a.level}: ratio {len(packed) / n:.3f} ok={ok} "
      f"{min(ts):.2f} ms -> {n / min(ts) / 1e6:.1f} GB/s", flush=True)
if os.environ.get("ZSTD_CPU"):
    import time
    for th in (1, 16):
        t = time.perf_counter()
        r, out = O.decompress_chunks(packed, cs, n, "zstd", a.chunk, threads=th if th > 1 else 0)
        dt = time.perf_counter() - t
        print(f"reference zstd 1.5.2 decode on the host, {th} thread(s): {n / dt / 1e6:.0f} MB/s (ok={r == n})", flush=True)
