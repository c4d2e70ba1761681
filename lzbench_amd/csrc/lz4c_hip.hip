// lzbench_amd/csrc/lz4c_hip.hip -- LZ4 block compressor (v3) for gfx950, bit-exact with lz4 1.9.3.
//
// Same greedy parse as the reference (lz4/lz4.c:851-1240) and as the v1 kernel
// (lz4_hip.hip), organised so that one sequence costs one batch of ~150 wave instructions and
// one dependent global-memory round trip:
//
//   * input ring: 1 KiB of the chunk around the parse front lives in LDS, filled ahead of
//     the front by LDS-DMA (buffer_load ... lds).  Probe hashing, the ip-2 insert, ip-side
//     catch-up / match-length bytes and literal bytes read LDS.
//   * speculative candidate window: the 4-byte candidate compare loads 24 bytes
//     [cand-4, cand+20) per lane; the hit lane's window (parked in 32 B of LDS) answers
//     catch-up (<= 4 bytes, lz4.c:1019) and the first 12 bytes of LZ4_count (lz4.c:603-626)
//     lane-parallel, without a second round trip.
//   * deferred, branch-free emission: a sequence's bytes are stored while the next batch's
//     candidate loads are in flight.
//   * fast probe plan: with acceleration 1 the first 65 probes of a search step by 1, so a
//     batch that starts a search (or re-tests a match end) is simply positions base+lane.
// Long catch-ups / matches / literal runs beyond the windows take lane-parallel slow paths.
#include "common.h"

namespace lz4v3 {

// optional per-kernel event counters (debug builds of the launch only; nullptr in production)
#define LZ_STAT(i, v) do { if (stats && lane == 0) atomicAdd(&stats[i], (unsigned long long)(v)); } while (0)
// debug-only phase clock (s_memtime) accumulated per wave
#define LZ_T(k) do { if (stats) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); ph[k] += t_ - tlast; tlast = t_; } } while (0)

constexpr int kMinMatch = 4;
constexpr int kMfLimit = 12;
constexpr int kLastLiterals = 5;
constexpr int kMinLength = 13;
constexpr int kRing = 1024;           // bytes of LDS input ring per wave
constexpr int kAhead = 704;           // keep the ring filled this far past the batch front
constexpr int kRT = 16;               // probe lanes of a re-test batch

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ int64_t step_prefix(int64_t M) {
    int64_t q = M >> 6, r = M & 63;
    return 32 * q * (q - 1) + r * q;
}

template <bool kSmall>
struct Table {
    LDSA uint32_t* raw;
    __device__ __forceinline__ uint32_t get(uint32_t h) const {
        if (kSmall) return ((volatile const LDSA uint16_t*)raw)[h];
        return ((volatile const LDSA uint32_t*)raw)[h];
    }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const {
        if (kSmall) ((volatile LDSA uint16_t*)raw)[h] = (uint16_t)v; else ((volatile LDSA uint32_t*)raw)[h] = v;
    }
};

template <bool kSmall>
__device__ __forceinline__ uint32_t hash_of(uint32_t w32, uint32_t b4) {
    if (kSmall) return (w32 * 2654435761u) >> 19;
    const uint64_t v = (uint64_t)w32 | ((uint64_t)b4 << 32);
    return (uint32_t)(((v << 24) * 889523592379ull) >> 52);
}

// LDS ring over descriptor offsets X = p + sh: holds [fill - kRing, fill).
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

__device__ __forceinline__ int ext_len_bytes(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

// Emit one sequence (has_match) or the final literal run at op. Each lane computes its
// byte of the sequence without branching; literal bytes come from the ring when it holds
// them. Returns the new op.
__device__ __forceinline__ int emit_seq(const Bytes& in, const Ring& R, const Bytes& out, int op, int anchor, int lit,
                                        bool has_match, int off, int ml, int lane) {
    const int lx = ext_len_bytes(lit);
    const int mx = has_match ? ext_len_bytes(ml) : 0;
    const int lit0 = 1 + lx, lit1 = lit0 + lit;            // literal bytes at [lit0, lit1)
    const int total = lit1 + (has_match ? 2 + mx : 0);
    const uint32_t token = ((uint32_t)min(lit, 15) << 4) | (has_match ? (uint32_t)min(ml, 15) : 0u);
    const uint32_t lrem = (uint32_t)((lit - 15) % 255), mrem = (uint32_t)((ml - 15) % 255);
    const bool lit_in_ring = R.has(anchor, anchor + lit);
    if (!lit_in_ring && lit > 2 * LZH_WAVE) {
        // long literal run: header, bulk copy, trailer
        if (lane == 0) out.st8(op, token);
        for (int b = lane; b < lx; b += LZH_WAVE) out.st8(op + 1 + b, b == lx - 1 ? lrem : 255u);
        copy_span(in, anchor, out, op + lit0, lit, lane, LZH_WAVE);
        if (has_match) {
            if (lane < 2) out.st8(op + lit1 + lane, lane ? ((uint32_t)off >> 8) : ((uint32_t)off & 0xffu));
            for (int b = lane; b < mx; b += LZH_WAVE) out.st8(op + lit1 + 2 + b, b == mx - 1 ? mrem : 255u);
        }
        return op + total;
    }
    for (int base = 0; base < total; base += LZH_WAVE) {
        const int t = base + lane;
        const int lp = anchor + t - lit0;
        const bool inlit = t >= lit0 && t < lit1;
        uint32_t lb = 0;
        if (lit_in_ring) lb = R.byte(lp);
        else if (inlit) lb = in.b(lp);
        const int u = t - (lit1 + 2);
        uint32_t v = token;
        v = (t >= 1 && t < lit0) ? (t == lx ? lrem : 255u) : v;
        v = inlit ? lb : v;
        v = t == lit1 ? ((uint32_t)off & 0xffu) : v;
        v = t == lit1 + 1 ? ((uint32_t)off >> 8) : v;
        v = (u >= 0) ? (u == mx - 1 ? mrem : 255u) : v;
        if (t < total) out.st8(op + t, v);
    }
    return op + total;
}

// M-side byte of the hit lane's window: spec index si (0..23) of the six uniform dwords
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

template <bool kSmall>
__device__ void compress_chunk(const Bytes& in, int n, const Bytes& out, int acc, LDSA uint32_t* tab, LDSA uint32_t* ringw,
                               LDSA uint32_t* specw, uint32_t* out_size, unsigned long long* stats) {
    (void)specw;
    const int lane = threadIdx.x;
    Table<kSmall> T{tab};
    if (n <= 0) {
        if (lane == 0) out.st8(0, 0);
        if (lane == 0) *out_size = 1;
        return;
    }
    {
        LDSA uint32_t* t4 = (LDSA uint32_t*)tab;
#pragma unroll
        for (int i = 0; i < 16; i++) lds_zero16(t4 + 4 * (i * LZH_WAVE + lane));
    }
    Ring R{ringw, in.sh, 0};
    const int endX = n + in.sh + 8;
    for (int s = 0; s < kRing / 256 && R.fill < endX; s++) R.refill(in.r, lane);
    wait_vm();
    wave_lds_fence();

    int op = 0, anchor = 0;
    bool pend = false;                       // deferred sequence
    int p_anchor = 0, p_lit = 0, p_off = 0, p_ml = 0;

    if (n >= kMinLength) {
        const int mfl1 = n - kMfLimit + 1;
        const int mlimit = n - kLastLiterals;
        const int64_t a64 = (int64_t)acc << 6;
        const int hb = kSmall ? 4 : 5;

        {
            const uint32_t h0 = hash_of<kSmall>(R.u32(0), R.byte(4));
            if (lane == 0) T.put(h0, 0);
            wave_lds_fence();
        }
        int ip = 1, s = 1, k0 = 0;
        bool retest = false;
        uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
        uint64_t tlast = stats ? __builtin_amdgcn_s_memtime() : 0;

        for (int guard = 0; guard < 4 * n + 64; guard++) {
            LZ_T(5);
            // ---- probe plan: lane -> position, validity (forwardIp <= mflimitPlusOne)
            const bool fast = acc == 1 && k0 == 0;
            // in a fast re-test batch lane 63 carries the ip-2 table fill (lz4.c:1146) instead of
            // a probe; it is written before any probe reads the table
            const bool ins63 = fast && retest;
            // a re-test batch probes only kRT lanes: the first hit after a match is almost always
            // within a few positions, and idle lanes issue no candidate loads
            int p;
            bool valid, term;
            if (fast) {
                p = (retest ? ip : s) + lane;            // re-test ip, then search ip+1.. step 1
                const bool act = !retest || lane < kRT;
                valid = act && p + 1 <= mfl1;
                term = act && p + 1 > mfl1;
                if (ins63 && lane == 63) { p = ip - 2; valid = false; term = false; }
            } else {
                int64_t pp, nxt;
                if (retest && lane == 0) {
                    pp = ip;
                    nxt = (int64_t)ip + 1;
                } else {
                    const int k = retest ? lane - 1 : k0 + lane;
                    const int64_t o = k == 0 ? 0 : 1 + step_prefix(a64 + k - 1) - step_prefix(a64);
                    const int64_t st = k == 0 ? 1 : (a64 + k - 1) >> 6;
                    pp = (int64_t)s + o;
                    nxt = pp + st;
                }
                valid = nxt <= mfl1;
                term = !valid;
                p = valid ? (int)pp : 0;
            }
            const uint64_t vmask = ballot(valid);
            const uint64_t tmask = ballot(term);
            const int front = ins63 ? ip - 2 : rdlanei(p, 0);
            const int pmax = vmask ? rdlanei(p, 63 - __builtin_clzll(vmask)) : front;
            LZ_STAT(0, 1);
            LZ_STAT(2, fast ? 1 : 0);

            // ---- hash (ring when it covers the batch)
            uint32_t pw, b4 = 0;
            if (R.has(front - 4, pmax + hb + 8)) {
                pw = R.u32(p);
                if (!kSmall) b4 = R.byte(p + 4);
            } else if (kSmall) {
                LZ_STAT(9, 1);
                pw = in.w32(p);
            } else {
                const uint64_t v = in.w40(p);
                pw = (uint32_t)v;
                b4 = (uint32_t)(v >> 32);
            }
            const uint32_t h = hash_of<kSmall>(pw, b4);
            if (ins63 && lane == 63) T.put(h, (uint32_t)(ip - 2));
            else if (retest && !fast) {   // general plan: the ip-2 fill happened before the batch
            }
            const uint32_t old = T.get(h);
            if (valid) T.put(h, (uint32_t)p);
            wave_lds_fence();
            const uint32_t back = T.get(h);
            // lanes whose table write lost to another lane of the batch (same slot)
            const uint64_t losers = ballot(valid && back != (uint32_t)p);
            uint32_t cand = old;
            LZ_T(0);
            // ---- speculative candidate window [cand-4, cand+20)
            int cX = (valid ? (int)cand : 0) + in.sh;
            int cA = (cX & ~3) - 4;
            uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0, d4 = 0, d5 = 0;
            if (valid) {
                d0 = ld_b32(in.r, cA); d1 = ld_b32(in.r, cA + 4); d2 = ld_b32(in.r, cA + 8);
                d3 = ld_b32(in.r, cA + 12); d4 = ld_b32(in.r, cA + 16); d5 = ld_b32(in.r, cA + 20);
            }
            // ---- deferred emission of the previous sequence (stores overlap the loads above)
            if (pend) {
                op = emit_seq(in, R, out, op, p_anchor, p_lit, true, p_off, p_ml, lane);
                pend = false;
            }
            // ---- keep the ring ahead of the batch front
            {
                const int target = min(front + in.sh + kAhead, endX + 256);
                for (int r = 0; r < 4 && R.fill < target; r++) { R.refill(in.r, lane); LZ_STAT(12, 1); }
            }
            LZ_T(1);
            wait_vm();
            wave_lds_fence();
            LZ_T(2);

            bool ok = valid && __builtin_amdgcn_alignbyte(d2, d1, (uint32_t)cX & 3u) == pw;
            if (!kSmall) ok = ok && (cand + 65535u >= (uint32_t)p);
            uint64_t hits = ballot(ok);
            const int fi = ffs64(tmask);
            int fh = ffs64(hits);
            bool found = hits != 0;
            int L = found ? fh : fi - 1;
            uint64_t upto = L < 0 ? 0ull : (L >= 63 ? ~0ull : ((2ull << L) - 1ull));
            // exact resolution is needed only if two lanes <= L share a slot; any such pair has
            // a loser <= L, and for small L the pair test is a few cross-lane compares
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
                // keep writes of lanes <= L: winners above L restore, then lanes <= L re-assert
                if (valid && lane > L && back == (uint32_t)p) T.put(h, old);
                if (losers & upto) {
                    wave_lds_fence();
                    if (lane <= L) T.put(h, (uint32_t)p);
                }
            } else {
                LZ_STAT(1, 1);
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
                cA = (cX & ~3) - 4;
                if (valid) {
                    d0 = ld_b32(in.r, cA); d1 = ld_b32(in.r, cA + 4); d2 = ld_b32(in.r, cA + 8);
                    d3 = ld_b32(in.r, cA + 12); d4 = ld_b32(in.r, cA + 16); d5 = ld_b32(in.r, cA + 20);
                }
                ok = valid && __builtin_amdgcn_alignbyte(d2, d1, (uint32_t)cX & 3u) == pw;
                if (!kSmall) ok = ok && (cand + 65535u >= (uint32_t)p);
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
                if (tmask) break;                                      // ran past mflimit
                if (retest) { retest = false; s = ip + 1; k0 = fast ? kRT - 1 : LZH_WAVE - 1; }
                else k0 += LZH_WAVE;
                continue;
            }
            wave_lds_fence();

            // ---- hit at P with candidate M; one lane-parallel compare answers catch-up
            // (lanes 0..3: P-1-j vs M-1-j, lz4.c:1019) and the match length from P+4 (lanes 4..:
            // P+4+k vs M+4+k, LZ4_count lz4.c:603-626).  Catch-up back bk moves both starts but
            // not the match end: count(P-bk+4) = bk + count(P+4).
            LZ_T(3);
            const int P = rdlanei(p, fh);
            const int M = rdlanei((int)cand, fh);
            const uint32_t e0 = rdlane(d0, fh), e1 = rdlane(d1, fh), e2 = rdlane(d2, fh), e3 = rdlane(d3, fh),
                           e4 = rdlane(d4, fh), e5 = rdlane(d5, fh);
            LZ_STAT(3, 1);
            LZ_STAT(4, fh);
            const int sbase = ((M + in.sh) & 3) + 4;           // window index of byte M
            const int kmax = 20 - sbase;                        // count bytes the window holds (13..16)
            const int maxb = min(P - anchor, M);
            const int blim = min(maxb, 4);
            int qpos, si;
            bool act;
            if (lane < 4) { qpos = P - 1 - lane; si = sbase - 1 - lane; act = lane < blim; }
            else { const int k = lane - 4; qpos = P + 4 + k; si = sbase + 4 + k; act = k < kmax; }
            const bool rok = R.has(P - 4, P + 4 + 16);
            uint32_t pb = 0;
            if (rok) pb = R.byte(qpos);
            else if (act) pb = in.b(qpos);
            const bool eq = act && pb == spec_byte(si & 31, e0, e1, e2, e3, e4, e5);
            const uint64_t em = ballot(eq);
            int bk = ffs64(~em & 0xfull);
            if (bk > blim) bk = blim;
            int cnt = ffs64((~(em >> 4) & ((1ull << kmax) - 1ull)) | (1ull << kmax));
            if (bk == 4 && maxb > 4) {
                LZ_STAT(5, 1);
                int ip2 = P - 4, m2 = M - 4;
                for (int it = 0; it < (1 << 12); it++) {
                    const int mb2 = min(ip2 - anchor, m2);
                    if (mb2 <= 0) break;
                    const bool e2b = lane < mb2 && in.b(ip2 - 1 - lane) == in.b(m2 - 1 - lane);
                    const int b = ffs64(ballot(!e2b));
                    ip2 -= b;
                    m2 -= b;
                    if (b < LZH_WAVE) break;
                }
                bk = P - ip2;
            }
            const int a = P + kMinMatch;                        // count start before catch-up
            if (cnt >= kmax && a + cnt < mlimit) {
                LZ_STAT(6, 1);
                for (int it = 0; it < (1 << 10) && a + cnt < mlimit; it++) {
                    const int o = cnt + 4 * lane;
                    const uint32_t x = in.w32(a + o) ^ in.w32(M + kMinMatch + o);
                    const uint64_t ne = ballot(x != 0);
                    if (ne) {
                        const int l = ffs64(ne);
                        cnt += 4 * l + (__builtin_ctz(rdlane(x, l)) >> 3);
                        break;
                    }
                    cnt += 4 * LZH_WAVE;
                }
            }
            cnt = min(cnt, mlimit - a);
            const int P2 = P - bk;
            const int lit = P2 - anchor;
            const int ml = bk + cnt;
            LZ_STAT(7, bk > 0 ? 1 : 0);
            LZ_STAT(10, lit);
            LZ_STAT(11, ml);
            pend = true;
            p_anchor = anchor; p_lit = lit; p_off = P - M; p_ml = ml;

            ip = a + cnt;                                       // = P2 + 4 + ml
            anchor = ip;
            if (ip >= mfl1) break;
            if (acc != 1) {   // general plan: fill table at ip-2 now (fast plan: lane 63 next batch)
                uint32_t w, bb = 0;
                if (R.has(ip - 6, ip + 8)) { w = R.u32(ip - 2); if (!kSmall) bb = R.byte(ip + 2); }
                else { const uint64_t v = in.w40(ip - 2); w = (uint32_t)v; bb = (uint32_t)(v >> 32); }
                const uint32_t hm2 = hash_of<kSmall>(w, bb);
                if (lane == 0) T.put(hm2, (uint32_t)(ip - 2));
                wave_lds_fence();
            }
            LZ_T(4);
            retest = true;
            s = ip + 1;
            k0 = 0;
        }
        for (int k = 0; k < 6; k++) LZ_STAT(16 + k, ph[k]);
    }
    if (pend) op = emit_seq(in, R, out, op, p_anchor, p_lit, true, p_off, p_ml, lane);
    op = emit_seq(in, R, out, op, anchor, n - anchor, false, 0, 0, lane);
    if (lane == 0) *out_size = (uint32_t)op;
}

}  // namespace lz4v3

extern "C" __global__ void __launch_bounds__(64)
lzh_lz4_compress_v2_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size, int acc,
                           uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t chunk0,
                           unsigned long long* stats) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4096 + 256 + 8];
    const uint64_t chunk = (uint64_t)blockIdx.x + chunk0;
    const uint64_t off = chunk * chunk_size;
    if (off >= n_total && !(n_total == 0 && chunk == 0)) return;
    const int n = (int)min(chunk_size, n_total - off);
    const uint64_t readable = min<uint64_t>(in_readable - off, (uint64_t)n + 64);
    Bytes rin, rout;
    rin.init(in + off, readable);
    rout.init(stage + chunk * stride, stride);
    if (n < 65547) lz4v3::compress_chunk<true>(rin, n, rout, acc, (LDSA uint32_t*)lds, (LDSA uint32_t*)lds + 4096, (LDSA uint32_t*)lds + 4096 + 256, csizes + chunk, stats);
    else lz4v3::compress_chunk<false>(rin, n, rout, acc, (LDSA uint32_t*)lds, (LDSA uint32_t*)lds + 4096, (LDSA uint32_t*)lds + 4096 + 256, csizes + chunk, stats);
}

#include "launch.h"
hipError_t lzh_launch_lz4_compress_v2(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                      int acc, uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks,
                                      hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(lzh_lz4_compress_v2_kernel, dim3(nchunks), dim3(64), 0, s, in, n_total, in_readable,
                       chunk_size, acc, stage, stride, csizes, 0u, (unsigned long long*)nullptr);
    return hipGetLastError();
}

// debug: run the v2 kernel with event counters (16 x u64 device buffer)
extern "C" int lzh_debug_lz4_stats(const void* d_in, uint64_t n, uint64_t in_readable, uint64_t chunk_size, int acc,
                                   void* d_stage, uint32_t* d_csizes, unsigned long long* d_stats, void* stream) {
    const uint64_t k = (n + chunk_size - 1) / chunk_size;
    const uint64_t stride = ((chunk_size + chunk_size / 255 + 16 + 16) + 255) / 256 * 256;
    hipLaunchKernelGGL(lzh_lz4_compress_v2_kernel, dim3((unsigned)k), dim3(64), 0, (hipStream_t)stream,
                       (const uint8_t*)d_in, n, in_readable, chunk_size, acc, (uint8_t*)d_stage, stride, d_csizes, 0u,
                       d_stats);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
