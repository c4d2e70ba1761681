"""tools/zstdc_stats.py -- phase clocks of the zstd entropy kernel (lane 0 of every frame, stamps 16..22).
Needs a -DLZH_ZSTDC_STATS=1 build: tools/exp_build.sh zst "-DLZH_ZSTDC_STATS=1", then
LZH_LIB=build/exp/zst/liblzbench_hip.so python tools/zstdc_stats.py [corpus] [chunk_kib] [mib]"""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch, lzbench_amd as L
lib = L.lib()
f = lib.lzh_debug_zstdc_stats
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_int]
corpus = sys.argv[1] if len(sys.argv) > 1 else "mixed"
chunk = int(sys.argv[2] if len(sys.argv) > 2 else 128) << 10
n = int(sys.argv[3] if len(sys.argv) > 3 else 256) << 20
host = L.datagen(corpus, n, seed=12345)
d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda"); d_in[:n].copy_(torch.from_numpy(host))
dc = L.DeviceCodec("zstd", n, chunk, level=1)
dc.compress(d_in)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 24)()
assert f(buf, 1) == 0
dc.compress_kernel_only(d_in)
torch.cuda.synchronize()
assert f(buf, 0) == 0
v = list(buf)
blocks = max(n // chunk, 1)
ze = {16: "lit_histo", 17: "huf_tree", 18: "huf_streams", 19: "seq_histo", 20: "fse_tables", 21: "seq_chains", 22: "seq_packing"}
zt = sum(v[i] for i in ze) or 1
fr = max(v[5], 1)
print(corpus, chunk >> 10, "KiB: match kernel per frame: clocks search %.0f match %.0f fills %.0f; batches %.0f, "
      "sequences %.0f; clocks per batch %.0f, per sequence (match + fills) %.0f" % (
          v[0] / fr, v[1] / fr, v[2] / fr, v[3] / fr, v[4] / fr, v[0] / max(v[3], 1), (v[1] + v[2]) / max(v[4], 1)))
print(corpus, chunk >> 10, "KiB:", "entropy clocks/block %.0f:" % (zt / blocks), {k: "%.1f%%" % (100 * v[i] / zt) for i, k in ze.items()})
