// lzbench_amd/csrc/snappyc_hip.hip -- snappy raw compressor (v2) for gfx950, bit-exact with
// snappy 1.1.8.  Same parse as v1 (snappy_hip.hip; reference snappy/snappy.cc:510-681, framing
// :1043-1111) with the structure of the LZ4 v4 kernel (lz4c_hip.hip):
//   * 1 KiB LDS input ring per wave filled ahead by LDS-DMA: probe hashing, the ip-1 insert,
//     ip-side match bytes and literal bytes read LDS;
//   * speculative candidate window [cand, cand+24) per probe lane: the hit lane's window answers
//     the first ~16 bytes of FindMatchLength (snappy-internal.h:100-224) lane-parallel;
//   * re-test batches (after a copy: insert ip-1, re-test ip, snappy.cc:652-656) use 16 probe
//     lanes plus lane 63 for the ip-1 insert; search batches use 64 lanes along the 16-unrolled /
//     skip>>5 schedule (snappy.cc:558-611);
//   * exact in-batch slot-collision handling only when two lanes up to the first hit collide;
//   * deferred, branch-free emission of literal + copy (EmitLiteral / EmitCopy, :342-443).
#include "common.h"

namespace snv2 {

#define SN_STAT(i, v) do { if (stats && lane == 0) atomicAdd(&stats[i], (unsigned long long)(v)); } while (0)

constexpr int kRing = 1024;
constexpr int kAhead = 704;
constexpr int kRT = 16;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

struct Table {
    LDSA uint16_t* t;
    __device__ __forceinline__ uint32_t get(uint32_t h) const { return ((volatile const LDSA uint16_t*)t)[h]; }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const { ((volatile LDSA uint16_t*)t)[h] = (uint16_t)v; }
};

struct Ring {
    LDSA uint32_t* w;
    int sh;
    int fill;
    __device__ __forceinline__ bool has(int p0, int p1) const { return p0 + sh >= fill - kRing && p1 + sh <= fill; }
    __device__ __forceinline__ uint32_t dword(int a) const {
        return ((volatile const LDSA uint32_t*)w)[(a >> 2) & (kRing / 4 - 1)];
    }
    __device__ __forceinline__ uint32_t u32(int p) const {
        const int X = p + sh, a = X & ~3;
        return __builtin_amdgcn_alignbyte(dword(a + 4), dword(a), (uint32_t)X & 3u);
    }
    __device__ __forceinline__ uint32_t byte(int p) const {
        return ((volatile const LDSA uint8_t*)w)[(p + sh) & (kRing - 1)];
    }
    __device__ __forceinline__ void refill(rsrc_t r, int lane) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(w + ((fill & (kRing - 1)) >> 2)), 4, fill + 4 * lane,
                                                 0, 0, 0);
        fill += 256;
    }
};

__device__ __forceinline__ int log2floor_u(uint32_t v) { return 31 - __builtin_clz(v); }

__device__ __forceinline__ uint32_t table_size_for(uint32_t n) {
    if (n > (1u << 14)) return 1u << 14;
    if (n < (1u << 8)) return 1u << 8;
    return 2u << log2floor_u(n - 1);
}

// u after i steps of u -> u + (u >> 5), one constant-step segment at a time (i <= 64 here)
__device__ __forceinline__ uint32_t skip_walk(uint32_t u, int i) {
    for (int it = 0; it < 80 && i > 0; it++) {
        const uint32_t m = u >> 5;
        uint32_t t = (32u * (m + 1) - u + m - 1) / m;
        if (t > (uint32_t)i) t = (uint32_t)i;
        u += t * m;
        i -= (int)t;
    }
    return u;
}

// emit [literal of len lit from position src][copy (off, mlen) if mlen > 0] at op; returns op
__device__ __forceinline__ int emit_seq(const Bytes& in, const Ring& R, const Bytes& out, int op, int src, int lit,
                                        uint32_t off, int mlen, int lane) {
    // literal header (snappy.cc:342-383)
    int hl = 0;
    uint32_t tag = 0, nm1 = (uint32_t)(lit - 1);
    int cnt = 0;
    if (lit > 0) {
        if (nm1 < 60) { hl = 1; tag = nm1 << 2; }
        else { cnt = (log2floor_u(nm1) >> 3) + 1; hl = 1 + cnt; tag = (uint32_t)(59 + cnt) << 2; }
    }
    // copy pieces (snappy.cc:385-443)
    int k = 0, has60 = 0, rem = mlen;
    if (mlen >= 12) {
        k = mlen >= 68 ? (mlen - 68) / 64 + 1 : 0;
        rem = mlen - 64 * k;
        if (rem > 64) { has60 = 1; rem -= 60; }
    }
    const bool c1 = rem < 12 && off < 2048u;
    const int pre = 3 * (k + has60);
    const int cb = mlen > 0 ? pre + (c1 ? 2 : 3) : 0;
    const int lit0 = hl, lit1 = hl + lit, total = lit1 + cb;
    const uint32_t lo = off & 0xffu, hi = (off >> 8) & 0xffu;
    const bool lit_in_ring = R.has(src, src + lit);
    if (!lit_in_ring && lit > 2 * LZH_WAVE) {
        if (lane == 0) out.st8(op, tag);
        if (lane >= 1 && lane < hl) out.st8(op + lane, (nm1 >> (8 * (lane - 1))) & 0xffu);
        copy_span(in, src, out, op + lit0, lit, lane, LZH_WAVE);
        for (int base = 0; base < cb; base += LZH_WAVE) {
            const int t = base + lane;
            uint32_t v;
            if (t < pre) {
                const int piece = t / 3, b = t - 3 * piece;
                v = b == 0 ? ((piece < k) ? (2u | (63u << 2)) : (2u | (59u << 2))) : (b == 1 ? lo : hi);
            } else {
                const int b = t - pre;
                if (c1) v = b == 0 ? (1u | ((uint32_t)(rem - 4) << 2) | ((off >> 8) << 5)) : lo;
                else v = b == 0 ? (2u | ((uint32_t)(rem - 1) << 2)) : (b == 1 ? lo : hi);
            }
            if (t < cb) out.st8(op + lit1 + t, v);
        }
        return op + total;
    }
    for (int base = 0; base < total; base += LZH_WAVE) {
        const int t = base + lane;
        const int lp = src + t - lit0;
        const bool inlit = t >= lit0 && t < lit1;
        uint32_t lb = 0;
        if (lit_in_ring) lb = R.byte(lp);
        else if (inlit) lb = in.b(lp);
        uint32_t v = tag;
        v = (t >= 1 && t < hl) ? ((nm1 >> (8 * (t - 1))) & 0xffu) : v;
        v = inlit ? lb : v;
        const int ct = t - lit1;
        if (ct >= 0) {
            uint32_t cv;
            if (ct < pre) {
                const int piece = ct / 3, b = ct - 3 * piece;
                cv = b == 0 ? ((piece < k) ? (2u | (63u << 2)) : (2u | (59u << 2))) : (b == 1 ? lo : hi);
            } else {
                const int b = ct - pre;
                if (c1) cv = b == 0 ? (1u | ((uint32_t)(rem - 4) << 2) | ((off >> 8) << 5)) : lo;
                else cv = b == 0 ? (2u | ((uint32_t)(rem - 1) << 2)) : (b == 1 ? lo : hi);
            }
            v = cv;
        }
        if (t < total) out.st8(op + t, v);
    }
    return op + total;
}

__device__ __forceinline__ uint32_t spec_byte(int si, uint32_t e0, uint32_t e1, uint32_t e2, uint32_t e3, uint32_t e4,
                                              uint32_t e5) {
    const int q = si >> 2;
    uint32_t v = e0;
    v = q == 1 ? e1 : v;
    v = q == 2 ? e2 : v;
    v = q == 3 ? e3 : v;
    v = q == 4 ? e4 : v;
    v = q == 5 ? e5 : v;
    return (v >> (8 * (si & 3))) & 0xffu;
}

// one fragment in[0, fn) appended at op
__device__ int compress_fragment(const Bytes& in, int fn, const Bytes& out, int op, LDSA uint16_t* tab,
                                 LDSA uint32_t* ringw, unsigned long long* stats) {
    const int lane = threadIdx.x;
    Table T{tab};
    const uint32_t tsize = table_size_for((uint32_t)fn);
    const int shift = 32 - log2floor_u(tsize);
    {
        LDSA uint32_t* t4 = (LDSA uint32_t*)tab;
        const int nvec = (int)(tsize * 2 / 16);
        for (int i = lane; i < nvec; i += LZH_WAVE) lds_zero16(t4 + 4 * i);
    }
    Ring R{ringw, in.sh, 0};
    const int endX = fn + in.sh + 8;
    for (int s = 0; s < kRing / 256 && R.fill < endX; s++) R.refill(in.r, lane);
    wait_vm();
    wave_lds_fence();

    int next_emit = 0;
    bool pend = false;
    int p_src = 0, p_lit = 0, p_ml = 0;
    uint32_t p_off = 0;
    if (fn >= 15) {
        const int ip_limit = fn - 15;
        bool retest = false;
        int rt = 0, q0 = 1, t0 = 0;
        bool U = ip_limit - q0 >= 16;
        int ci0 = 0, cq0 = U ? q0 + 16 : q0;
        uint32_t cu0 = U ? 48u : 32u;
        for (int guard = 0; guard < 4 * fn + 64; guard++) {
            // ---- probe plan
            int p = 0;
            bool valid = false, term = false;
            int ci = -1;                 // checked-probe index of this lane (-1: not a checked probe)
            uint32_t u = 0;
            const bool ins63 = retest;   // lane 63 inserts ip-1 before the re-test reads
            if (retest && lane == 0) {
                p = rt;
                valid = true;
            } else if (ins63 && lane == 63) {
                p = rt - 1;
            } else if (!retest || lane < kRT) {
                const int t = retest ? lane - 1 : t0 + lane;
                if (U && t < 16) {
                    p = q0 + t;
                    valid = true;
                } else {
                    ci = U ? t - 16 : t;
                    u = skip_walk(cu0, ci - ci0);
                    const int64_t pp = (int64_t)cq0 + (int64_t)(u - cu0);
                    valid = pp + (int64_t)(u >> 5) <= ip_limit;
                    term = !valid;
                    p = valid ? (int)pp : 0;
                }
            }
            const uint64_t vmask = ballot(valid);
            const uint64_t tmask = ballot(term);
            const int front = ins63 ? rt - 1 : rdlanei(p, 0);
            const int pmax = vmask ? rdlanei(p, 63 - __builtin_clzll(vmask)) : front;
            SN_STAT(0, 1);

            uint32_t pw;
            if (R.has(front - 4, pmax + 12)) pw = R.u32(p);
            else { SN_STAT(9, 1); pw = in.w32(p); }
            const uint32_t h = (pw * 0x1e35a7bdu) >> shift;
            if (ins63 && lane == 63) T.put(h, (uint32_t)(rt - 1));
            const uint32_t old = T.get(h);
            if (valid) T.put(h, (uint32_t)p);
            wave_lds_fence();
            const uint32_t back = T.get(h);
            const uint64_t losers = ballot(valid && back != (uint32_t)p);
            uint32_t cand = old;
            int cX = (valid ? (int)cand : 0) + in.sh;
            int cA = cX & ~3;
            uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0, d4 = 0, d5 = 0;
            if (valid) {
                d0 = ld_b32(in.r, cA); d1 = ld_b32(in.r, cA + 4); d2 = ld_b32(in.r, cA + 8);
                d3 = ld_b32(in.r, cA + 12); d4 = ld_b32(in.r, cA + 16); d5 = ld_b32(in.r, cA + 20);
            }
            if (pend) {
                op = emit_seq(in, R, out, op, p_src, p_lit, p_off, p_ml, lane);
                pend = false;
            }
            {
                const int target = min(front + in.sh + kAhead, endX + 256);
                for (int r = 0; r < 4 && R.fill < target; r++) R.refill(in.r, lane);
            }
            wait_vm();
            wave_lds_fence();

            bool ok = valid && __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)cX & 3u) == pw;
            uint64_t hits = ballot(ok);
            const int fi = ffs64(tmask);
            int fh = ffs64(hits);
            bool found = hits != 0;
            int L = found ? fh : fi - 1;
            uint64_t upto = L < 0 ? 0ull : (L >= 63 ? ~0ull : ((2ull << L) - 1ull));
            bool exact = false;
            if (losers & upto) {
                if (L <= 7) {
                    bool pr = false;
#pragma unroll
                    for (int d = 1; d <= 7; d++) {
                        const uint32_t hv = lane_gather(h, lane >= d ? lane - d : lane);
                        pr = pr || (d <= lane && lane <= L && hv == h);
                    }
                    exact = ballot(pr) != 0;
                } else {
                    exact = true;
                }
            }
            if (!exact) {
                if (valid && lane > L && back == (uint32_t)p) T.put(h, old);
                if (losers & upto) {
                    wave_lds_fence();
                    if (lane <= L) T.put(h, (uint32_t)p);
                }
            } else {
                SN_STAT(1, 1);
                if (valid) T.put(h, old);
                wave_lds_fence();
                uint64_t pending = losers;
                uint64_t grp = 1ull << lane;
                int prev = -1;
                for (int it = 0; it < LZH_WAVE && pending; it++) {
                    const int l = ffs64(pending);
                    const uint32_t hv = rdlane(h, l);
                    const bool mine = valid && h == hv;
                    const uint64_t m = ballot(mine);
                    pending &= ~m;
                    if (mine) {
                        grp = m;
                        const uint64_t below = m & ((1ull << lane) - 1ull);
                        if (below) prev = 63 - __builtin_clzll(below);
                    }
                }
                const uint32_t ppos = lane_gather((uint32_t)p, prev < 0 ? lane : prev);
                if (prev >= 0) cand = ppos;
                cX = (valid ? (int)cand : 0) + in.sh;
                cA = cX & ~3;
                if (valid) {
                    d0 = ld_b32(in.r, cA); d1 = ld_b32(in.r, cA + 4); d2 = ld_b32(in.r, cA + 8);
                    d3 = ld_b32(in.r, cA + 12); d4 = ld_b32(in.r, cA + 16); d5 = ld_b32(in.r, cA + 20);
                }
                ok = valid && __builtin_amdgcn_alignbyte(d1, d0, (uint32_t)cX & 3u) == pw;
                hits = ballot(ok);
                fh = ffs64(hits);
                found = hits != 0;
                L = found ? fh : fi - 1;
                upto = L < 0 ? 0ull : (L >= 63 ? ~0ull : ((2ull << L) - 1ull));
                if (valid && lane <= L) {
                    const uint64_t later = grp & ~((2ull << lane) - 1ull) & upto;
                    if (!later) T.put(h, (uint32_t)p);
                }
            }
            if (!found) {
                wave_lds_fence();
                if (tmask) break;                         // search exhausted: remainder from next_emit
                // advance the checked-probe reference past this batch's last probe lane
                const int last = retest ? kRT - 1 : 63;
                const int cl = rdlanei(ci, last);
                if (cl >= 0) {
                    const uint32_t ul = rdlane(u, last);
                    const int ql = rdlanei(p, last);
                    ci0 = cl + 1;
                    cq0 = ql + (int)(ul >> 5);
                    cu0 = ul + (ul >> 5);
                }
                if (retest) { retest = false; t0 = kRT - 1; }
                else t0 += LZH_WAVE;
                continue;
            }
            wave_lds_fence();
            // ---- copy at P from candidate M: FindMatchLength(M+4, P+4, fn), first bytes from the
            // window (lanes k: P+4+k vs M+4+k), the rest lane-parallel from memory
            const int P = rdlanei(p, fh);
            const int M = rdlanei((int)cand, fh);
            const uint32_t e0 = rdlane(d0, fh), e1 = rdlane(d1, fh), e2 = rdlane(d2, fh), e3 = rdlane(d3, fh),
                           e4 = rdlane(d4, fh), e5 = rdlane(d5, fh);
            SN_STAT(3, 1);
            const int sbase = (M + in.sh) & 3;                 // window index of byte M
            const int kmax = 20 - sbase;                        // bytes M+4.. the window holds (17..20)
            const int a = P + 4;
            const bool rok = R.has(a, a + 20);
            const bool act = lane < kmax;
            uint32_t pb = 0;
            if (rok) pb = R.byte(a + lane);
            else if (act) pb = in.b(a + lane);
            const bool eq = act && pb == spec_byte((sbase + 4 + lane) & 31, e0, e1, e2, e3, e4, e5);
            const uint64_t em = ballot(eq);
            int len = ffs64((~em & ((1ull << kmax) - 1ull)) | (1ull << kmax));
            if (len >= kmax && a + len < fn) {
                SN_STAT(6, 1);
                for (int it = 0; it < (1 << 11) && a + len < fn; it++) {
                    const int o = len + 4 * lane;
                    const uint32_t x = in.w32(a + o) ^ in.w32(M + 4 + o);
                    const uint64_t ne = ballot(x != 0);
                    if (ne) {
                        const int l = ffs64(ne);
                        len += 4 * l + (__builtin_ctz(rdlane(x, l)) >> 3);
                        break;
                    }
                    len += 4 * LZH_WAVE;
                }
            }
            len = min(len, fn - a);
            const int matched = 4 + len;
            pend = true;
            p_src = next_emit; p_lit = P - next_emit; p_off = (uint32_t)(P - M); p_ml = matched;
            const int ip = P + matched;
            next_emit = ip;
            if (ip >= ip_limit) break;
            retest = true;
            rt = ip;
            q0 = ip + 1;
            t0 = 0;
            U = ip_limit - q0 >= 16;
            ci0 = 0;
            cq0 = U ? q0 + 16 : q0;
            cu0 = U ? 48u : 32u;
        }
    }
    if (pend) op = emit_seq(in, R, out, op, p_src, p_lit, p_off, p_ml, lane);
    if (next_emit < fn) op = emit_seq(in, R, out, op, next_emit, fn - next_emit, 0, 0, lane);
    wave_lds_fence();
    return op;
}

}  // namespace snv2

extern "C" __global__ void __launch_bounds__(64)
lzh_snappy_compress_v2_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                              uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t chunk0,
                              unsigned long long* stats) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[(1 << 13) + 256];
    const int lane = threadIdx.x;
    const uint64_t chunk = (uint64_t)blockIdx.x + chunk0;
    const uint64_t off = chunk * chunk_size;
    if (off >= n_total && !(n_total == 0 && chunk == 0)) return;
    const uint32_t n = (uint32_t)min(chunk_size, n_total - off);
    Bytes rout;
    rout.init(stage + chunk * stride, stride);
    int op = 0;
    {   // varint32 uncompressed length (snappy.cc:1047-1050)
        uint32_t v = n;
        int nb = 1;
        while (v >= 128) { v >>= 7; nb++; }
        if (lane < nb) rout.st8(lane, ((n >> (7 * lane)) & 0x7fu) | (lane + 1 < nb ? 0x80u : 0u));
        op = nb;
    }
    for (uint32_t fpos = 0; fpos < n; fpos += 65536u) {
        const int fn = (int)min(65536u, n - fpos);
        const uint64_t readable = min<uint64_t>(in_readable - off - fpos, (uint64_t)fn + 64);
        Bytes rin;
        rin.init(in + off + fpos, readable);
        op = snv2::compress_fragment(rin, fn, rout, op, (LDSA uint16_t*)lds, (LDSA uint32_t*)lds + (1 << 13), stats);
    }
    if (lane == 0) csizes[chunk] = (uint32_t)op;
}

#include "launch.h"
hipError_t lzh_launch_snappy_compress_v2(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                         uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks,
                                         hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(lzh_snappy_compress_v2_kernel, dim3(nchunks), dim3(64), 0, s, in, n_total, in_readable,
                       chunk_size, stage, stride, csizes, 0u, (unsigned long long*)nullptr);
    return hipGetLastError();
}
