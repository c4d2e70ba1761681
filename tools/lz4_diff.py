"""tools/lz4_diff.py -- first differing LZ4 sequence between the HIP compressor and the oracle.
usage: python tools/lz4_diff.py [corpus] [chunk_kib] [acc] [MiB] [seed]"""
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
mib = int(sys.argv[4]) if len(sys.argv) > 4 else 1
seed = int(sys.argv[5]) if len(sys.argv) > 5 else 7
d = L.datagen(corpus, mib << 20, seed)
p, cs = L.compress_chunks(d, codec, chunk, acc)
op, ocs = O.compress_chunks(d, codec, chunk, acc, threads=16)
bad = np.nonzero(cs != ocs)[0]
if len(bad) == 0 and not (p == op).all():   # same sizes, different bytes
    offs = np.concatenate([[0], np.cumsum(cs.astype(np.int64))])
    first = int(np.nonzero(p != op)[0][0])
    bad = np.array([int(np.searchsorted(offs, first, side="right") - 1)])
print("bad chunks", len(bad), bad[:10])
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
