"""tools/dec_debug.py -- locate the first decoder mismatch (lz4) and list the sequences around it."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch, lzbench_amd as L


def lz4_seqs(b):
    ip, op, out = 0, 0, []
    while ip < len(b):
        t = b[ip]; ip += 1
        lit = t >> 4
        if lit == 15:
            while True:
                s = b[ip]; ip += 1; lit += s
                if s != 255: break
        lp = ip; ip += lit
        if ip >= len(b):
            out.append((op, lit, 0, 0, lp)); break
        off = b[ip] | (b[ip + 1] << 8); ip += 2
        ml = t & 15
        if ml == 15:
            while True:
                s = b[ip]; ip += 1; ml += s
                if s != 255: break
        ml += 4
        out.append((op, lit, off, ml, lp))
        op += lit + ml
    return out


for corpus in sys.argv[1:] or ["text", "json", "mixed"]:
    n = 8 << 20
    host = L.datagen(corpus, n, seed=7)
    d = torch.zeros(n + 256, dtype=torch.uint8, device="cuda"); d[:n].copy_(torch.from_numpy(host))
    dc = L.DeviceCodec("lz4", n, 65536)
    dc.compress(d); dc.decompress(); torch.cuda.synchronize()
    out = dc.out[:n].cpu().numpy()
    st = dc.status.cpu().numpy()
    bad = np.nonzero(out != host)[0]
    print(corpus, "mismatching bytes", len(bad), "bad status", int((st < 0).sum()))
    if len(bad) == 0: continue
    p = int(bad[0]); c = p // 65536; rel = p - c * 65536
    offs = dc.offsets.cpu().numpy(); cs = dc.csizes.cpu().numpy()
    blk = dc.packed[int(offs[c]):int(offs[c]) + int(cs[c])].cpu().numpy().tobytes()
    print(" chunk", c, "rel", rel, "status", st[c], "bad in chunk", int(((bad >= c * 65536) & (bad < (c + 1) * 65536)).sum()))
    e = host[c * 65536 + rel - 8: c * 65536 + rel + 24]; g = out[c * 65536 + rel - 8: c * 65536 + rel + 24]
    print(" exp", bytes(e)); print(" got", bytes(g))
    print(" bad rel offsets", (bad[:20] - c * 65536).tolist())
    for s in lz4_seqs(blk):
        if s[0] + s[1] + s[3] >= rel - 64 and s[0] <= rel + 64:
            print("  seq op=%d lit=%d off=%d ml=%d  [lit %d..%d) [match %d..%d)" % (s[0], s[1], s[2], s[3], s[0], s[0] + s[1], s[0] + s[1], s[0] + s[1] + s[3]))
