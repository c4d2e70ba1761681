"""tools/sn_clk.py -- phase clocks of the snappy parse kernel's run batches (an experiment build with
-DLZH_SN_CLK, tools/exp_build.sh snclk "-DLZH_SN_CLK"; run with LZH_LIB=build/exp/snclk/liblzbench_hip.so).
usage: python tools/sn_clk.py [corpus] [chunk_kib] [MiB]"""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch, lzbench_amd as L
corpus = sys.argv[1] if len(sys.argv) > 1 else "json"
chunk = (int(sys.argv[2]) if len(sys.argv) > 2 else 64) << 10
n = (int(sys.argv[3]) if len(sys.argv) > 3 else 512) << 20
lib = L.lib()
f = lib.lzh_debug_snappy_clocks
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_int]
host = L.datagen(corpus, n, seed=12345)
d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda"); d_in[:n].copy_(torch.from_numpy(host))
dc = L.DeviceCodec("snappy", n, chunk)
buf = np.zeros(16, np.uint64)
f(buf.ctypes.data, 1)
dc.compress_stage(d_in, 1)
torch.cuda.synchronize()
f(buf.ctypes.data, 1)
names = ["P side+hash+table+loads+claim", "record stores", "slot groups", "load wait", "eval+resolve", "records",
         "restore+state", "search batches"]
tot = sum(int(x) for x in buf[:8]) or 1
frags = int(buf[8]) or 1
print(corpus, chunk >> 10, "KiB: clocks per fragment %.0f" % (tot / frags),
      {names[i]: "%.1f%%" % (100 * int(buf[i]) / tot) for i in range(8)})
