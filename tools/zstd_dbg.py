"""Debug: decode specific reference zstd frames on the GPU and report the first differing byte,
with the frame's block structure (headers parsed here in Python, test infrastructure)."""
import os, sys
import numpy as np
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "tests"))
import torch
import lzbench_amd as L, oracle_lib as O
from test_gpu_zstd import gpu_decode

def blocks(f):
    fhd = f[4]; single = (fhd >> 5) & 1; fcsf = fhd >> 6
    p = 5 + (0 if single else 1) + [0, 1, 2, 4][fhd & 3]
    fsz = [1 if single else 0, 2, 4, 8][fcsf]
    p += fsz
    out = []
    while True:
        bh = f[p] | (f[p+1] << 8) | (f[p+2] << 16); p += 3
        last, typ, bsz = bh & 1, (bh >> 1) & 3, bh >> 3
        info = dict(type=typ, bsz=bsz)
        if typ == 2:
            b0 = f[p]; lt = b0 & 3; sf = (b0 >> 2) & 3
            info.update(ltype=lt, sf=sf)
            if lt <= 1:
                hsz = 1 if (sf & 1) == 0 else (2 if sf == 1 else 3)
                rs = (b0 >> 3) if hsz == 1 else ((b0 >> 4) + (f[p+1] << 4) + ((f[p+2] << 12) if hsz == 3 else 0))
                sp = p + hsz + (rs if lt == 0 else 1)
            else:
                hsz = 3 if sf <= 1 else (4 if sf == 2 else 5); bits = 10 if sf <= 1 else (14 if sf == 2 else 18)
                h = int.from_bytes(bytes(f[p:p+hsz]), "little"); rs = (h >> 4) & ((1 << bits) - 1); cs = (h >> (4 + bits)) & ((1 << bits) - 1)
                info.update(lcs=cs, huf_hdr=f[p + hsz]); sp = p + hsz + cs
            info.update(rs=rs)
            ns = f[sp]; q = sp + 1
            if ns >= 128:
                if ns == 255: ns = f[q] + (f[q+1] << 8) + 0x7F00; q += 2
                else: ns = ((ns - 128) << 8) + f[q]; q += 1
            info.update(nseq=ns)
            if ns: info.update(modes=(f[q] >> 6, (f[q] >> 4) & 3, (f[q] >> 2) & 3))
        out.append(info)
        p += bsz if typ != 1 else 1
        if last: break
    return out

for kind, n, chunk, level in [("binary", 100003, 262144, 3), ("binary", 100003, 262144, 1), ("binary", 100000, 262144, 3),
                              ("binary", 131072, 131072, 3), ("binary", 100003, 131072, 3), ("text", 100003, 262144, 3)]:
    data = L.datagen(kind, n, 5)
    packed, cs = O.compress_chunks(data, "zstd", chunk, level)
    st, out = gpu_decode(torch, packed, cs, n, chunk)
    d = np.nonzero(out != data)[0]
    print(kind, n, chunk, level, "status", st, "ndiff", len(d), "first", d[:8], flush=True)
    if len(d):
        print("  blocks", blocks(packed[:cs[0]]))
        i = d[0]; print("  got", out[i-4:i+12], "\n  exp", data[i-4:i+12])
