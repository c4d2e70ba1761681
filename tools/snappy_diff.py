"""tools/snappy_diff.py -- first differing snappy tag between the HIP compressor and the oracle.
usage: python tools/snappy_diff.py [corpus] [chunk_kib]"""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import lzbench_amd as L, oracle_lib as O


def tags(b):
    """(output position, kind, length, offset) per tag of one snappy stream."""
    i, pos, out = 0, 0, []
    while b[i] & 0x80: i += 1
    i += 1
    while i < len(b):
        c = b[i]; i += 1
        k = c & 3
        if k == 0:
            ln = (c >> 2) + 1
            if ln > 60:
                nb = ln - 60; ln = int.from_bytes(bytes(b[i:i + nb]), "little") + 1; i += nb
            out.append((pos, "L", ln, 0)); i += ln; pos += ln
        else:
            if k == 1: ln = ((c >> 2) & 7) + 4; off = ((c >> 5) << 8) | b[i]; i += 1
            elif k == 2: ln = (c >> 2) + 1; off = b[i] | (b[i + 1] << 8); i += 2
            else: ln = (c >> 2) + 1; off = int.from_bytes(bytes(b[i:i + 4]), "little"); i += 4
            out.append((pos, "C", ln, off)); pos += ln
    return out


corpus = sys.argv[1] if len(sys.argv) > 1 else "text"
chunk = (int(sys.argv[2]) if len(sys.argv) > 2 else 64) << 10
d = L.datagen(corpus, 1 << 20, 7)
p, cs = L.compress_chunks(d, "snappy", chunk)
op, ocs = O.compress_chunks(d, "snappy", chunk)
go = np.concatenate([[0], np.cumsum(cs)]).astype(np.int64)
oo = np.concatenate([[0], np.cumsum(ocs)]).astype(np.int64)
shown = 0
for c in range(len(cs)):
    a = p[go[c]:go[c + 1]].tobytes(); b = op[oo[c]:oo[c + 1]].tobytes()
    if a == b: continue
    ta, tb = tags(a), tags(b)
    k = next(i for i in range(min(len(ta), len(tb))) if ta[i] != tb[i])
    print(f"chunk {c}: first differing tag {k}: gpu {ta[max(0,k-3):k+3]}\n   ref {tb[max(0,k-3):k+3]}")
    pos = tb[k][0]
    base = c * chunk
    print("   input around", pos, bytes(d[base + pos - 20: base + pos + 40]))
    frag = (pos // 65536) * 65536
    def h(q):
        v = int.from_bytes(bytes(d[base + q: base + q + 4]), "little")
        return ((v * 0x1e35a7bd) & 0xffffffff) >> 18
    for q in range(pos - 2, pos + 6):
        same = [r for r in range(frag, q) if h(r) == h(q)]
        print(f"   pos {q} hash {h(q)} earlier same-hash positions {same[-6:]}")
    shown += 1
    if shown >= 4: break
