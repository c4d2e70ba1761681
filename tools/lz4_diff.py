"""tools/lz4_diff.py -- first differing LZ4 sequence between the HIP compressor and the oracle.
usage: python tools/lz4_diff.py [corpus] [chunk_kib] [acc]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import lzbench_amd as L, oracle_lib as O


def seqs(b):
    out, i, pos = [], 0, 0
    while i < len(b):
        t = b[i]; i += 1
        lit = t >> 4
        if lit == 15:
            while True:
                s = b[i]; i += 1; lit += s
                if s != 255: break
        i += lit
        if i >= len(b):
            out.append((pos, lit, 0, 0)); break
        off = b[i] | (b[i + 1] << 8); i += 2
        ml = t & 15
        if ml == 15:
            while True:
                s = b[i]; i += 1; ml += s
                if s != 255: break
        ml += 4
        out.append((pos, lit, off, ml))
        pos += lit + ml
    return out


corpus = sys.argv[1] if len(sys.argv) > 1 else "text"
chunk = (int(sys.argv[2]) if len(sys.argv) > 2 else 64) << 10
acc = int(sys.argv[3]) if len(sys.argv) > 3 else 1
codec = "lz4" if acc == 1 else "lz4fast"
d = L.datagen(corpus, 1 << 20, 7)
p, cs = L.compress_chunks(d, codec, chunk, acc)
op, ocs = O.compress_chunks(d, codec, chunk, acc)
bad = np.nonzero(cs != ocs)[0]
print("bad chunks", bad[:10])
shown = 0
for c in bad[:3]:
    go = int(np.sum(cs[:c])); oo = int(np.sum(ocs[:c]))
    g = seqs(p[go:go + cs[c]].tobytes()); o = seqs(op[oo:oo + ocs[c]].tobytes())
    for k, (a, b) in enumerate(zip(g, o)):
        if a != b:
            print(f"chunk {c} seq {k}: gpu (pos,lit,off,ml)={a} ref={b}; prev ref {o[max(0,k-3):k]}")
            base = c * chunk
            pos = b[0]
            print("   bytes around:", bytes(d[base + pos: base + pos + b[1] + 24]))
            break
