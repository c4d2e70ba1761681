"""tools/dec_stats.py -- event counters and phase clocks of the LZ4 / snappy group decoder.
Needs a -DLZH_DEC_STATS=1 build: tools/exp_build.sh decst "-DLZH_DEC_STATS=1", then
LZH_LIB=build/exp/decst/liblzbench_hip.so python tools/dec_stats.py [codec] [corpus]"""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch, lzbench_amd as L
lib = L.lib()
f = lib.lzh_debug_dec_stats
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_int]
codec = sys.argv[1] if len(sys.argv) > 1 else "lz4"
corpus = sys.argv[2] if len(sys.argv) > 2 else "text"
chunk = int(os.environ.get("STATS_KIB", "64")) << 10
n = int(os.environ.get("STATS_MIB", "256")) << 20
host = L.datagen(corpus, n, seed=12345)
d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda"); d_in[:n].copy_(torch.from_numpy(host))
dc = L.DeviceCodec(codec, n, chunk)
dc.compress(d_in)
torch.cuda.synchronize()
buf = (C.c_ulonglong * 16)()
assert f(buf, 1) == 0
dc.decompress()
torch.cuda.synchronize()
assert f(buf, 0) == 0
v = list(buf)
k = max(v[11], 1)
names = ["groups", "members", "passes", "passes_k1", "rounds", "far_passes", "checked", "group_bytes"]
print(codec, corpus, "per chunk:", {names[i]: round(v[i] / k, 1) for i in range(8)})
print("  members/group %.2f  bytes/group %.1f  passes/group %.2f" % (v[1] / max(v[0], 1), v[7] / max(v[0], 1), v[2] / max(v[0], 1)))
tot = v[12] or 1
print("  clocks/chunk %.0f: parse %.1f%%  emit %.1f%%  checked %.1f%%  other %.1f%%" % (
    tot / k, 100 * v[8] / tot, 100 * v[9] / tot, 100 * v[10] / tot, 100 * (tot - v[8] - v[9] - v[10]) / tot))
