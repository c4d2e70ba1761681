"""zstd decode check on the GPU: reference-compressed frames (oracle/_ref, zstd 1.5.2) of several
corpora / chunk sizes / levels through lzh_decompress_async(LZH_CODEC_ZSTD); prints per-config
status histogram and first mismatch, plus a kernel timing on a larger input."""
import os, sys, time
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import torch
import lzbench_amd as L, oracle_lib as O

def run(data, chunk, level):
    packed, cs = O.compress_chunks(data, "zstd", chunk, level)
    n = len(data)
    dc = L.DeviceCodec("zstd", n, chunk)
    d_packed = torch.zeros(len(packed) + 256, dtype=torch.uint8, device="cuda")
    d_packed[:len(packed)].copy_(torch.from_numpy(packed))
    d_cs = torch.from_numpy(cs.astype(np.int32)).cuda()
    dc.decompress(packed=d_packed, csizes=d_cs)
    torch.cuda.synchronize()
    st = dc.status[:dc.k].cpu().numpy()
    out = dc.out[:n].cpu().numpy()
    exp = np.array([min(chunk, n - i * chunk) for i in range(dc.k)])
    bad = np.nonzero(st != exp)[0]
    ok = len(bad) == 0 and (out == data).all()
    msg = ""
    if not ok:
        if len(bad):
            u, c = np.unique(st[bad], return_counts=True)
            msg = f"{len(bad)}/{dc.k} chunks bad, status codes {dict(zip(u.tolist(), c.tolist()))}"
        else:
            d = np.nonzero(out != data)[0]
            msg = f"bytes differ first at {d[0]} (chunk {d[0] // chunk}, off {d[0] % chunk}), {len(d)} bytes"
    return ok, msg, len(packed) / n, (dc, d_packed, d_cs)

tot_bad = 0
for kind in sys.argv[1:] or ["text", "json", "random", "binary", "mixed"]:
    data = L.datagen(kind, 4 << 20, 11)
    for chunk, level in [(131072, 1), (65536, 1), (262144, 1), (131072, 3), (131072, 6), (131072, 19)]:
        t = time.time()
        ok, msg, ratio, _ = run(data, chunk, level)
        tot_bad += not ok
        print(f"{kind:7s} b{chunk >> 10:4d} l{level:2d} ratio {ratio:.3f} {'OK' if ok else 'FAIL ' + msg} {time.time() - t:.1f}s", flush=True)
print("BAD", tot_bad, flush=True)
# timing: 256 MiB text, -b128, level 1
data = L.datagen("text", 256 << 20, 3)
ok, msg, ratio, (dc, d_packed, d_cs) = run(data, 131072, 1)
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ts = []
for _ in range(3):
    s.record(); dc.decompress(packed=d_packed, csizes=d_cs); e.record(); torch.cuda.synchronize()
    ts.append(s.elapsed_time(e))
print(f"timing 256 MiB text -b128 l1: ok={ok} {min(ts):.2f} ms -> {len(data) / min(ts) / 1e6:.1f} GB/s", flush=True)
