"""tools/dec_dbg.py -- first wrong output bytes of the GPU decoder on small corpora (decoder debugging).
usage: python tools/dec_dbg.py [MiB]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import lzbench_amd as L
mib = float(sys.argv[1]) if len(sys.argv) > 1 else 1
n = int(mib * (1 << 20))
for codec, corpus, ck in (("lz4", "text", 65536), ("lz4", "json", 65536), ("lz4", "mixed", 65536),
                          ("snappy", "mixed", 262144), ("snappy", "text", 65536)):
    data = L.datagen(corpus, n, seed=12345)
    packed, cs = L.compress_chunks(data, codec, ck)
    out = L.decompress_chunks(packed, cs, n, codec, ck)
    bad = np.nonzero(out != data)[0]
    print(f"{codec} {corpus}: {len(bad)} wrong bytes", flush=True)
    if len(bad):
        chunks = np.unique(bad // ck)
        print("  chunks", chunks[:10], "first", bad[:12], flush=True)
        b = int(bad[0])
        lo = max(b - 8, 0)
        print("  want", data[lo:b + 12].tolist(), "\n  got ", out[lo:b + 12].tolist(), flush=True)
        c = int(chunks[0]); cb = bad[bad // ck == c] - c * ck
        print(f"  chunk {c}: {len(cb)} wrong, offsets in chunk {cb[:16].tolist()}", flush=True)
