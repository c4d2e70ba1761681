"""tools/rows_diff.py -- first chunks where the batched rows (lzbench_hip_compress_batch, ngpus logical shards)
differ from the reference chunk loop, and whether each differing chunk's sub-batch recompressed alone matches.
usage: python tools/rows_diff.py codec chunk_kib MiB corpus level ngpus"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import lzbench_amd as L, oracle_lib as O
codec, ck, mib, corpus, level, ng = sys.argv[1], int(sys.argv[2]) << 10, int(sys.argv[3]), sys.argv[4], int(sys.argv[5]), int(sys.argv[6])
n = mib << 20
data = L.datagen(corpus, n, seed=12345)
p, cs = L.compress_chunks(data, codec, ck, level, ngpus=ng)
rp, rcs = O.compress_chunks(data, codec, ck, level, use_ref=True, threads=16)
print("sizes equal", bool((cs == rcs).all()), "packed equal", len(p) == len(rp) and bool((p == rp).all()), flush=True)
offs = np.concatenate([[0], np.cumsum(cs.astype(np.int64))])
roffs = np.concatenate([[0], np.cumsum(rcs.astype(np.int64))])
bad = [i for i in range(len(cs)) if cs[i] != rcs[i] or not (p[offs[i]:offs[i + 1]] == rp[roffs[i]:roffs[i + 1]]).all()]
print("bad chunks", len(bad), bad[:20], flush=True)
for i in bad[:3]:
    a, b = p[offs[i]:offs[i + 1]], rp[roffs[i]:roffs[i + 1]]
    d = np.nonzero(a != b)[0]
    print(f"chunk {i}: size {cs[i]}, {len(d)} bytes differ, first at {d[:8]} gpu {a[d[:8]]} ref {b[d[:8]]}", flush=True)
    one, ocs = L.compress_chunks(data[i * ck:(i + 1) * ck], codec, ck, level)
    print(f"   alone: equal to ref {len(one) == len(b) and bool((one == b).all())}", flush=True)
