"""tools/split_dbg.py -- the snappy split decode's layout (split flags, fragment descriptors, fragment
statuses) for the hand-built streams of tests/test_gpu_snappy_split.py (debugging)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import lzbench_amd as L
import test_gpu_snappy_split as T
rng = np.random.default_rng(7)
chunk = 131072
ss = []
s = T._Stream(); T._fill(s, rng, 65500, True); s.lit(rng.integers(0, 256, 100).astype(np.uint8).tobytes()); T._fill(s, rng, chunk, True); ss.append(s)
s = T._Stream(); T._fill(s, rng, 65536, True); s.copy(1000, 64); T._fill(s, rng, chunk, True); ss.append(s)
s = T._Stream(); T._fill(s, rng, 65536, True); s.lit(rng.integers(0, 256, 70).astype(np.uint8).tobytes()); T._fill(s, rng, chunk, True); ss.append(s)
streams = [x.bytes() for x in ss]
k = len(streams); n = k * chunk
blob = b"".join(streams)
d_packed = torch.zeros(len(blob) + 256, dtype=torch.uint8, device="cuda")
d_packed[: len(blob)].copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
d_cs = torch.tensor([len(x) for x in streams], dtype=torch.int32, device="cuda")
dc = L.DeviceCodec("snappy", n, chunk)
dc.decompress(packed=d_packed, csizes=d_cs)
torch.cuda.synchronize()
t = dc.dtemp.cpu().numpy()
F = 2
al = lambda v: (v + 255) & ~255
sb = al((k + 1) * 8)
desc = t[sb: sb + k * F * 32].view(np.uint32).reshape(k * F, 8)
fst = t[sb + al(k * F * 32): sb + al(k * F * 32) + k * F * 4].view(np.int32)
cfl = t[sb + al(k * F * 32) + al(k * F * 4): sb + al(k * F * 32) + al(k * F * 4) + k * 4].view(np.uint32)
print("lens", [len(x) for x in streams])
print("cflag", cfl.tolist())
print("desc (src lo, cs, ds, flags)", [(int(d[0]), int(d[4]), int(d[5]), int(d[6])) for d in desc])
print("fstat", fst.tolist())
print("status", dc.status[:k].cpu().numpy().tolist())
