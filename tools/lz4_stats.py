"""tools/lz4_stats.py -- event counters of the LZ4 compress kernel (debug launch)."""
import ctypes as C, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch, lzbench_amd as L
lib = L.lib()
f = lib.lzh_debug_lz4_stats
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_uint64, C.c_uint64, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
names = ["batches", "collision_batches", "slow_colliders", "sequences", "window_moved", "catchup_slow", "count_slow", "-",
         "-", "pside_from_memory", "-", "-", "refills", "-", "-", "-"]
for corpus in sys.argv[1:] or ["text", "json"]:
    n = int(os.environ.get("STATS_MIB", "512")) << 20
    host = L.datagen(corpus, n, seed=12345)
    d_in = torch.zeros(n + 256, dtype=torch.uint8, device="cuda"); d_in[:n].copy_(torch.from_numpy(host))
    acc = int(os.environ.get("STATS_ACC", "1"))
    dc = L.DeviceCodec("lz4fast" if acc > 1 else "lz4", n, 65536, level=acc)
    st = torch.zeros(32, dtype=torch.int64, device="cuda")
    assert f(d_in.data_ptr(), n, d_in.numel(), 65536, acc, dc.ctemp.data_ptr(), dc.csizes.data_ptr(), st.data_ptr(),
             torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    v = st.cpu().tolist()
    k = n // 65536
    print(corpus, {names[i]: round(v[i] / k, 2) for i in range(13) if names[i] != '-'}, "per chunk")
    clk = ["positions+pside+hash", "table+loads", "records", "load_wait", "eval+groups", "chain_resolve",
           "pr_state", "-", "table_restore", "other(stride,loop)", "links(in chain_resolve)", "walk(in chain_resolve)"]
    tot = sum(v[13:25]) or 1
    print("  clocks/chunk %.0f:" % (tot / k), {clk[i]: "%.1f%%" % (100 * v[13 + i] / tot) for i in range(12)})
