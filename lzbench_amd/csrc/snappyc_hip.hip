// lzbench_amd/csrc/snappyc_hip.hip -- snappy raw compressor for gfx950, bit-exact with snappy
// 1.1.8 (reference snappy/snappy.cc:510-681, framing :1043-1111).
//
// Run batches (the common case, as in the LZ4 kernel lz4c_hip.hip): the probe offsets of a
// snappy search are data independent -- 16 unrolled probes, then `skip >> 5` steps with skip
// from 48 (snappy.cc:558-611) give offsets 0..32, 34, 36, .., 62, 64, 67, .. from the search
// start (kPat0/kPat1) -- and after every copy snappy inserts ip-1, re-tests ip and searches from
// ip+1 (:640-672).  So a batch evaluates 64 consecutive positions speculatively (hash, LDS table
// claim/read-back, candidate window), resolves the chain of copies lane-parallel (per-lane match
// end + next hit under the probe pattern, scalar walk over the links, colliders verified against
// the resolved inserted set), and emits the batch's literals + copies lane-parallel under the
// next batch's loads.  Searches that run past offset 63 (sparse probes) and the last ~64
// positions of a fragment (exact termination) use the search batches below (v2):
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
#ifndef LZH_SN_PADLDS
#define LZH_SN_PADLDS 0
#endif
#ifndef LZH_SN_DPPEND   // the members' ends by a DPP running max (no lane_gather round trips)
#define LZH_SN_DPPEND 1
#endif
#ifndef LZH_SN_AMASK   // the resolve's hit set and probed set as uniform masks from single-compare ballots
#define LZH_SN_AMASK 1
#endif
#ifndef LZH_SN_SHR   // the next hit after a copy from A shifted down by the copy's end (no per-lane pattern)
#define LZH_SN_SHR 1
#endif
#ifndef LZH_SN_RESTORE2   // the table restore of a batch without slot collisions: no per-lane last-insert search
#define LZH_SN_RESTORE2 1
#endif
// phase clocks of the run batches (experiment builds with -DLZH_SN_CLK; tools/sn_clk.py): the time since the
// previous mark is charged to phase i, flushed per fragment into lzh_sn_clk_buf
#ifdef LZH_SN_CLK
__device__ unsigned long long lzh_sn_clk_buf[16];
#define SN_CLK(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); snclk[i] += t_ - snclk_last; snclk_last = t_; } while (0)
#else
#define SN_CLK(i) ((void)0)
#endif

constexpr int kRing = 1024;
constexpr int kAhead = 704;
constexpr int kRT = 16;
constexpr uint64_t kPat0 = 0x55555555ffffffffull;   // probe offsets 0..63 of a search (0..32, 34, .., 62)
constexpr uint64_t kPat1 = 0x2222222249249249ull;   // offsets 64..127 (64, 67, 70, ..)

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
    int ready;    // fill level known to have landed (refills are issued after a batch's load wait)
    bool on = true;    // (false: no LDS ring, every read goes to memory)
    bool mirror = false;   // the ring's first 32 bytes are mirrored past its end (reads never wrap)
    __device__ __forceinline__ bool has(int p0, int p1) const {
        return on && p0 + sh >= fill - kRing && p1 + sh <= ready;
    }
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
        if (!on) return;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(w + ((fill & (kRing - 1)) >> 2)), 4, fill + 4 * lane,
                                                 0, 0, 0);
        if (mirror && (fill & (kRing - 1)) == 0 && lane < 8)   // the same 32 bytes into the mirror
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(w + kRing / 4), 4, fill + 4 * lane, 0, 0, 0);
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

// Layout of one (literal, copy) pair, byte t of it per lane: EmitLiteral (snappy.cc:342-383:
// tag (len-1)<<2, or 60..63 followed by 1..4 length bytes) then EmitCopy (:385-443: 64-byte
// COPY_2 pieces while len >= 68, a 60-byte piece if len > 64, then COPY_1 when the last piece is
// < 12 long and the offset < 2048, else COPY_2).  lit may be 0 (no literal), mlen 0 (no copy).
struct SnapSeq {
    int hl, k, has60, rem, pre, cb, lit0, lit1, total;
    uint32_t tag, nm1, lo, hi, offv;
    bool c1;
    __device__ __forceinline__ SnapSeq(int lit, uint32_t off, int mlen) {
        hl = 0;
        tag = 0;
        nm1 = (uint32_t)(lit - 1);
        if (lit > 0) {
            if (nm1 < 60) { hl = 1; tag = nm1 << 2; }
            else { const int cnt = (log2floor_u(nm1) >> 3) + 1; hl = 1 + cnt; tag = (uint32_t)(59 + cnt) << 2; }
        }
        k = 0;
        has60 = 0;
        rem = mlen;
        if (mlen >= 12) {
            k = mlen >= 68 ? (mlen - 68) / 64 + 1 : 0;
            rem = mlen - 64 * k;
            if (rem > 64) { has60 = 1; rem -= 60; }
        }
        offv = off;
        c1 = rem < 12 && off < 2048u;
        pre = 3 * (k + has60);
        cb = mlen > 0 ? pre + (c1 ? 2 : 3) : 0;
        lit0 = hl;
        lit1 = hl + lit;
        total = lit1 + cb;
        lo = off & 0xffu;
        hi = (off >> 8) & 0xffu;
    }
    __device__ __forceinline__ uint32_t byte(int t, uint32_t lb) const {
        uint32_t v = tag;
        v = (t >= 1 && t < hl) ? ((nm1 >> ((8 * (t - 1)) & 31)) & 0xffu) : v;
        v = (t >= lit0 && t < lit1) ? lb : v;
        const int ct = t - lit1;
        if (ct >= 0) {
            uint32_t cv;
            if (ct < pre) {
                const int piece = ct / 3, b = ct - 3 * piece;
                cv = b == 0 ? ((piece < k) ? (2u | (63u << 2)) : (2u | (59u << 2))) : (b == 1 ? lo : hi);
            } else {
                const int b = ct - pre;
                if (c1) cv = b == 0 ? (1u | ((uint32_t)(rem - 4) << 2) | ((offv >> 8) << 5)) : lo;
                else cv = b == 0 ? (2u | ((uint32_t)(rem - 1) << 2)) : (b == 1 ? lo : hi);
            }
            v = cv;
        }
        return v;
    }
};

// Sequences found by one batch, one per member lane (the lane of the copy's start): literal
// start, literal length, offset, copy length, first output byte within the batch's output.
// Emitted lane-parallel under the next batch's loads.  (Plain locals: a struct here would be
// kept in scratch memory.)
#define SREC_DECL uint32_t rc_anc = 0, rc_lit = 0, rc_off = 0, rc_ml = 0, rc_st = 0; uint64_t rc_m = 0; int rc_tot = 0
#define SREC_EMIT() op = emit_recs(in, R, out, mark, op, rc_anc, rc_lit, rc_off, rc_ml, rc_st, rc_m, rc_tot, lane)
// kRec: the sequences leave as 8-byte records (copy start P in the chunk | copy length << 24 | offset << 48,
// chunk order; a literal-only record, copy length 0 at P = its end, ends a fragment) for
// lzh_snappy_emit_kernel instead of being laid out here; a record's literal run starts at the previous
// record's end
#define SREC_OUT()                                                                                 \
    do {                                                                                           \
        if (kRec) {                                                                                \
            const uint64_t rm_ = uni64(rc_m);   /* (wave-uniform: keep it in SGPRs) */             \
            if (rm_) {                                                                             \
                const int ri_ = nrec + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(rm_ >> 32),       \
                                           __builtin_amdgcn_mbcnt_lo((uint32_t)rm_, 0u));          \
                if (lane_on(rm_))                                                                  \
                    st_b64(recs, 8 * ri_, rc_lit | (rc_ml << 24), (rc_ml >> 8) | (rc_off << 16));    \
                nrec = unii(nrec + __builtin_popcountll(rm_));                                     \
            }                                                                                      \
        } else {                                                                                   \
            SREC_EMIT();                                                                           \
        }                                                                                          \
    } while (0)

__device__ __forceinline__ int emit_recs(const Bytes& in, const Ring& R, const Bytes& out, LDSA uint8_t* mark, int op,
                                         uint32_t anc, uint32_t lit, uint32_t off, uint32_t ml, uint32_t st,
                                         uint64_t mem, int tot, int lane) {
    if (mem == 0) return op;
    const int first = __builtin_ctzll(mem), last = 63 - __builtin_clzll(mem);
    const int a0 = rdlanei((int)anc, first), a1 = rdlanei((int)anc, last) + rdlanei((int)lit, last);
    if (tot <= 4 * LZH_WAVE && R.has(a0, a1)) {
        int carry = first;
        for (int pass = 0; pass * LZH_WAVE < tot; pass++) {
            const int pb = pass * LZH_WAVE, ob = pb + lane;
            // owner of output byte ob: the last member starting at or before it (start marks)
            mark[lane] = 0xff;
            wave_lds_fence();
            const int stl = (int)st;
            if (lane_on(mem) && stl >= pb && stl < pb + LZH_WAVE) mark[stl - pb] = (uint8_t)lane;
            wave_lds_fence();
            const int mv = (int)mark[lane];
            const uint64_t smask = ballot(mv != 0xff);
            const uint64_t le = smask & ((2ull << lane) - 1ull);
            const int own = (int)lane_gather((uint32_t)mv, le ? 63 - __builtin_clzll(le) : lane);
            const int k = le ? own : carry;
            carry = rdlanei(k, 63);
            const int a = (int)lane_gather(anc, k), l = (int)lane_gather(lit, k);
            const uint32_t o = lane_gather(off, k);
            const int m = (int)lane_gather(ml, k);
            const int t = ob - (int)lane_gather(st, k);
            const SnapSeq Q(l, o, m);
            const uint32_t lb = R.byte(a + t - Q.lit0);
            if (ob < tot) out.st8(op + ob, Q.byte(t, lb));
        }
        return op + tot;
    }
    for (uint64_t mm = mem; mm; mm &= mm - 1) {
        const int k = __builtin_ctzll(mm);
        op = emit_seq(in, R, out, op, rdlanei((int)anc, k), rdlanei((int)lit, k), rdlane(off, k), rdlanei((int)ml, k),
                      lane);
    }
    return op;
}

__device__ __forceinline__ uint32_t byte_ctz(uint32_t x) { return (uint32_t)__builtin_ctz(x) >> 3; }
__device__ __forceinline__ int ctz64v(uint64_t x) { return x ? __builtin_ctzll(x) : 64; }
__device__ __forceinline__ uint64_t lane_bits(int lo, int hi) {   // bits lo..hi (0 <= lo <= hi <= 63)
    return ((2ull << hi) - 1ull) & (~0ull << lo);
}
// lanes l (0..63) whose offset l - o from a search origin is a probe offset of the schedule
__device__ __forceinline__ uint64_t pat_from(int o) {
    if (o >= LZH_WAVE) return 0ull;
    if (o >= 0) return kPat0 << o;
    const int d = -o;
    if (d < LZH_WAVE) return (kPat0 >> d) | (kPat1 << (LZH_WAVE - d));
    if (d < 2 * LZH_WAVE) return kPat1 >> (d - LZH_WAVE);
    return 0ull;
}
// probes after a copy ending at lane e: the re-test at e, then the search from e+1
__device__ __forceinline__ uint64_t after_copy(int e) {
    if (e >= LZH_WAVE) return 0ull;
    return (1ull << e) | (e + 1 < LZH_WAVE ? kPat0 << (e + 1) : 0ull);
}

// P side: words at p, p+4, .., p+20 (ring); candidate side: 7 dwords from (c & ~3)
struct PS { uint32_t w, q1, q2, q3, q4, q5; };
__device__ __forceinline__ PS p_side(const Ring& R, const Bytes& in, bool ring, int p) {
    const int X = (ring ? p + R.sh : p + in.sh), A = X & ~3;
    const uint32_t s = (uint32_t)X & 3u;
    uint32_t a0, a1, a2, a3, a4, a5, a6;
    if (ring && R.mirror) {   // one base address, immediate offsets (the mirror absorbs the wrap)
        const volatile LDSA uint32_t* q = (const volatile LDSA uint32_t*)R.w + ((A & (kRing - 1)) >> 2);
        a0 = q[0]; a1 = q[1]; a2 = q[2]; a3 = q[3]; a4 = q[4]; a5 = q[5]; a6 = q[6];
    } else if (ring) {
        a0 = R.dword(A); a1 = R.dword(A + 4); a2 = R.dword(A + 8); a3 = R.dword(A + 12);
        a4 = R.dword(A + 16); a5 = R.dword(A + 20); a6 = R.dword(A + 24);
    } else {
        a0 = ld_b32(in.r, A); a1 = ld_b32(in.r, A + 4); a2 = ld_b32(in.r, A + 8); a3 = ld_b32(in.r, A + 12);
        a4 = ld_b32(in.r, A + 16); a5 = ld_b32(in.r, A + 20); a6 = ld_b32(in.r, A + 24);
    }
    PS v;
    v.w = __builtin_amdgcn_alignbyte(a1, a0, s);
    v.q1 = __builtin_amdgcn_alignbyte(a2, a1, s);
    v.q2 = __builtin_amdgcn_alignbyte(a3, a2, s);
    v.q3 = __builtin_amdgcn_alignbyte(a4, a3, s);
    v.q4 = __builtin_amdgcn_alignbyte(a5, a4, s);
    v.q5 = __builtin_amdgcn_alignbyte(a6, a5, s);
    return v;
}
// bytes matched after the first 4 (0..20) between two 24-byte windows
__device__ __forceinline__ int match_after4(const PS& a, uint32_t b1, uint32_t b2, uint32_t b3, uint32_t b4,
                                            uint32_t b5) {
    return first_diff20(a.q1 ^ b1, a.q2 ^ b2, a.q3 ^ b3, a.q4 ^ b4, a.q5 ^ b5);
}

// one fragment in[0, fn) appended at op (kRec: its records appended at nrec)
template <bool kRec>
__device__ int compress_fragment(const Bytes& in, int fn, const Bytes& out, int op, LDSA uint16_t* tab,
                                 LDSA uint32_t* ringw, LDSA uint8_t* mark, unsigned long long* stats, rsrc_t recs,
                                 int& nrec, int fbase) {
    const int lane = threadIdx.x;
    Table T{tab};
    const uint32_t tsize = table_size_for((uint32_t)fn);
    const int shift = 32 - log2floor_u(tsize);
    {
        LDSA uint32_t* t4 = (LDSA uint32_t*)tab;
        const int nvec = (int)(tsize * 2 / 16);
        for (int i = lane; i < nvec; i += LZH_WAVE) lds_zero16(t4 + 4 * i);
    }
    // (parse kernel: mirrored ring; without it and with every P side from memory 4-6 % slower, profiles/r05_snr;
    // with the register window of the LZ4 kernel instead -- 32 KiB, 5 waves per CU -- no faster, profiles/r06_f)
    Ring R{ringw, in.sh, 0, 0, true, kRec};
    const int endX = fn + in.sh + 8;
    for (int s = 0; s < kRing / 256 && R.fill < endX; s++) R.refill(in.r, lane);
    wait_vm();
    R.ready = R.fill;
    wave_lds_fence();

    int next_emit = 0;
    SREC_DECL;
#ifdef LZH_SN_CLK
    uint64_t snclk[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t snclk_last = __builtin_amdgcn_s_memtime();
#endif
    if (fn >= 15) {
        const int ip_limit = fn - 15;
        // run-batch state: batch base, search origin, pending re-test (-1: none)
        bool runm = true;
        int base = 1, org = 1, rt = -1;
        // search-batch state (see below)
        bool retest = false;
        int q0 = 1, t0 = 0;
        bool U = ip_limit - q0 >= 16;
        int ci0 = 0, cq0 = U ? q0 + 16 : q0;
        uint32_t cu0 = U ? 48u : 32u;
        for (int guard = 0; guard < 4 * fn + 64; guard++) {
            runm = unii(runm) != 0; retest = unii(retest) != 0; U = unii(U) != 0;
            base = unii(base); org = unii(org); rt = unii(rt); q0 = unii(q0); t0 = unii(t0);
            ci0 = unii(ci0); cq0 = unii(cq0); cu0 = uni(cu0); next_emit = unii(next_emit); op = unii(op);
            rc_tot = unii(rc_tot); R.fill = unii(R.fill); R.ready = unii(R.ready);
            SN_STAT(0, 1);
            if (runm && (base + LZH_WAVE + 8 > ip_limit || (rt < 0 && base - org >= LZH_WAVE))) {
                // leave run batches: sparse probes or close to ip_limit (exact termination below)
                runm = false;
                if (rt >= 0) {
                    retest = true;
                    q0 = rt + 1;
                    t0 = 0;
                } else {
                    const int d = base - org;                 // schedule probes before base
                    retest = false;
                    q0 = org;
                    t0 = d < LZH_WAVE ? __builtin_popcountll(kPat0 & ((1ull << d) - 1ull))
                                      : 48 + __builtin_popcountll(kPat1 & ((1ull << (d - LZH_WAVE)) - 1ull));
                }
                U = ip_limit - q0 >= 16;
                ci0 = 0;
                cq0 = U ? q0 + 16 : q0;
                cu0 = U ? 48u : 32u;
            }
            if (runm) {
                // ================= run batch: positions base..base+63 (all probes valid)
                const int p = base + lane;
                const uint64_t P0 = (rt >= 0 ? 2ull : 0ull) | pat_from(org - base);
                const uint64_t I0 = rt >= 0 ? 1ull : 0ull;              // lane 0 = rt-1 (inserted, snappy.cc:652)
                const bool ring = R.has(base, base + LZH_WAVE + 28);
                const PS ps = p_side(R, in, ring, p);
                const uint32_t h = (ps.w * 0x1e35a7bdu) >> shift;
                const uint32_t old = T.get(h);
                const uint32_t cand = old;
                uint32_t d0, d1, d2, d3, d4, d5, d6;
                {   // (the candidate window loads are issued before the claim round trip)
                    const int cX = (int)cand + in.sh, cA = cX & ~3;
                    d0 = ld_b32(in.r, cA); d1 = ld_b32(in.r, cA + 4); d2 = ld_b32(in.r, cA + 8);
                    d3 = ld_b32(in.r, cA + 12); d4 = ld_b32(in.r, cA + 16); d5 = ld_b32(in.r, cA + 20);
                    d6 = ld_b32(in.r, cA + 24);
                }
                T.put(h, (uint32_t)p);
                wave_lds_fence();
                const uint32_t back = T.get(h);
                const uint64_t losers = ballot(back != (uint32_t)p);
                SN_CLK(0);
                SREC_OUT();
                rc_m = 0;
                rc_tot = 0;
                SN_CLK(1);
                // (the slot groups and the collider pre-evaluation need no candidate bytes: they
                // run under the candidate loads)
                // slot groups: every lane of a slot read back the same claim winner
                const uint64_t below = (1ull << lane) - 1ull;
                uint64_t grp = 1ull << lane, coll = 0;
                int prev = -1;
                bool okp = false;
                uint64_t OKP = 0;                                        // (okp as a lane mask)
                int lep = 0;
                if (losers) {
                    SN_STAT(1, 1);
                    const uint32_t W = back - (uint32_t)base;
                    uint32_t ne0 = 0, ne1 = 0;                     // lanes whose winner differs in a bit
#pragma unroll
                    for (int b = 0; b < 6; b++) {
                        const uint64_t bm = ballot((W >> b) & 1u);
                        const uint32_t mine = (uint32_t)__builtin_amdgcn_sbfe((int)W, b, 1);   // 0 / ~0
                        ne0 |= (uint32_t)bm ^ mine;
                        ne1 |= (uint32_t)(bm >> 32) ^ mine;
                    }
                    grp = ~(((uint64_t)ne1 << 32) | ne0);
                    const uint64_t eb = grp & below;
                    prev = eb ? 63 - __builtin_clzll(eb) : -1;
                    coll = ballot(prev >= 0);
                    const int k = prev >= 0 ? prev : lane;
                    const uint32_t gw = lane_gather(ps.w, k);
                    lep = match_after4(ps, lane_gather(ps.q1, k), lane_gather(ps.q2, k), lane_gather(ps.q3, k),
                                       lane_gather(ps.q4, k), lane_gather(ps.q5, k));
                    okp = gw == ps.w;
                    OKP = ballot(gw == ps.w);
                }
                SN_CLK(2);
                wait_vm();
                R.ready = R.fill;
                wave_lds_fence();
                SN_CLK(3);
                {
                    const int target = min(base + in.sh + kAhead, endX + 256);
                    for (int r = 0; r < 4 && R.fill < target; r++) R.refill(in.r, lane);
                }
                const uint32_t cs = (uint32_t)(cand + in.sh) & 3u;
                const bool ok = __builtin_amdgcn_alignbyte(d1, d0, cs) == ps.w;
                const uint64_t OKM = ballot(ok);                         // (next to its compare: no VGPR trip)
                const int len = match_after4(ps, __builtin_amdgcn_alignbyte(d2, d1, cs),
                                             __builtin_amdgcn_alignbyte(d3, d2, cs),
                                             __builtin_amdgcn_alignbyte(d4, d3, cs),
                                             __builtin_amdgcn_alignbyte(d5, d4, cs),
                                             __builtin_amdgcn_alignbyte(d6, d5, cs));
                // resolve (as the LZ4 kernel): assume each collider's candidate is its closest
                // earlier slot member, walk, verify against the inserted set, repeat if needed
                int ak = prev;
                bool oke = prev >= 0 ? okp : ok;
                // (LZH_SN_AMASK) oke as a uniform mask: a ballot of the merged bool goes through a VGPR each round
                uint64_t Am = (coll & OKP) | (OKM & ~coll);
                uint32_t ce = prev >= 0 ? (uint32_t)(base + prev) : cand;
                int le = prev >= 0 ? lep : len;
                uint64_t Mm = 0, I = I0;
                int cn = 0, e = 0, eL = 0;
                int ejm = 0;                                             // (LZH_SN_DPPEND: the last round's running max)
                bool endp = false;
                for (int round = 0; round <= LZH_WAVE; round++) {
                    const uint64_t A = LZH_SN_AMASK ? uni64(Am) : ballot(oke);
                    cn = min(le, fn - (p + 4));                          // FindMatchLength limit (ip_end)
                    const bool lng = (LZH_SN_AMASK ? lane_on(A) : oke) && le == 20 && p + 24 < fn;
                    e = lane + 4 + cn;
                    // next hit at or after e on the pattern after a copy (LZH_SN_SHR: A shifted down by e, one 64-bit
                    // shift per lane, instead of the pattern built per lane)
                    constexpr uint64_t kAft = 1ull | (kPat0 << 1);
                    const int f = LZH_SN_SHR ? (e < LZH_WAVE ? e + ctz64v((A >> (e & 63)) & kAft) : LZH_WAVE)
                                             : ctz64v(A & after_copy(e));
                    const int link = (lng || p + 4 + cn >= ip_limit) ? 0x80 : f;
                    Mm = 0;
                    endp = false;
                    uint64_t E;
                    const uint64_t r0 = A & P0;
                    if (!r0) {
                        E = P0;
                    } else {
                        int sl = __builtin_ctzll(r0);
                        for (;;) {                                       // (links strictly increase)
                            int fs;
                            // one register for the walk, the last member the highest bit of Mm afterwards (members
                            // increase): 5 instructions a member (as the LZ4 kernel's walk)
                            fs = unii(sl);
                            Mm = uni64(Mm);
                            do {
                                asm("s_bitset1_b64 %0, %1" : "+s"(Mm) : "s"(fs));
                                fs = rdlanei(link, fs);
                            } while (fs < LZH_WAVE);
                            sl = 63 - __builtin_clzll(Mm);
                            if (fs != 0x80) break;
                            int es;
                            if (rdlane((uint32_t)lng, sl)) {             // copy runs past the window
                                SN_STAT(6, 1);
                                const int a = base + sl + 4, M = rdlanei((int)ce, sl);
                                int c = 20;
                                for (int it = 0; it < (1 << 11) && a + c < fn; it++) {
                                    const int o = c + 4 * lane;
                                    const uint32_t x = in.w32(a + o) ^ in.w32(M + 4 + o);
                                    const uint64_t ne = ballot(x != 0);
                                    if (ne) {
                                        const int l = ffs64(ne);
                                        c += 4 * l + (int)byte_ctz(rdlane(x, l));
                                        break;
                                    }
                                    c += 4 * LZH_WAVE;
                                }
                                c = min(c, fn - a);
                                es = sl + 4 + c;
                                cn = lane == sl ? c : cn;
                                e = lane == sl ? es : e;
                                fs = ctz64v(A & after_copy(es));
                            } else {
                                es = rdlanei(e, sl);
                            }
                            if (base + es >= ip_limit) { endp = true; break; }   // snappy.cc:646
                            if (fs >= LZH_WAVE) break;
                            sl = fs;
                        }
                        eL = rdlanei(e, sl);
                        // probed lanes: the initial plan up to the first member, then after each
                        // copy the re-test and the search pattern; ip-1 of each copy is inserted
                        if (LZH_SN_DPPEND) {
                            // end of the last member at or before the lane (0: none): members' ends
                            // increase along the chain (after_copy(e) holds lanes >= e only)
                            const bool mem = lane_on(Mm);
                            ejm = wave_incl_max(mem ? e : 0);
                            // (after_copy(ejm) at lane >= ejm is bit lane - ejm of kAfter: no per-lane 64-bit pattern)
                            constexpr uint64_t kAfter = 1ull | (kPat0 << 1);
                            if (LZH_SN_AMASK) {
                                // members; lanes before the first member on the initial plan; lanes at or past the
                                // last member's end on its pattern -- one compare per ballot, the rest scalar
                                const uint64_t Z = ballot(ejm == 0), GE = ballot(lane >= ejm),
                                               BT = ballot(((kAfter >> ((lane - ejm) & 63)) & 1ull) != 0ull);
                                const uint64_t below_eL = endp && eL < LZH_WAVE ? (1ull << eL) - 1ull : ~0ull;
                                E = (Mm | (Z & P0) | (~Z & GE & BT)) & below_eL;
                            } else {
                            bool pr;
                            if (mem) pr = true;
                            else if (ejm == 0) pr = lane_on(P0);
                            else pr = lane >= ejm && ((kAfter >> ((lane - ejm) & 63)) & 1ull);
                            E = ballot(pr && (!endp || lane < eL));
                            }
                            I = ballot(lane + 1 == ejm) & ~Mm;
                        } else {
                        const uint64_t mle = Mm & (below | (1ull << lane));
                        const int j = mle ? 63 - __builtin_clzll(mle) : lane;
                        const int ej = (int)lane_gather((uint32_t)e, j);
                        bool pr;
                        if (!mle) pr = lane_on(P0);
                        else if (lane == j) pr = true;
                        else pr = lane >= ej && ((after_copy(ej) >> lane) & 1ull);
                        E = ballot(pr && (!endp || lane < eL));
                        I = ballot(mle && lane != j && lane == ej - 1);
                        }
                    }
                    I = (Mm ? I : 0ull) | I0 | E;                          // (no stale bits from an earlier round)
                    if (!(coll & E)) break;
                    const uint64_t mk = grp & below & I;
                    const int kt = mk ? 63 - __builtin_clzll(mk) : -1;
                    const bool fix = lane_on(E) && kt != ak;
                    const uint64_t FX = ballot(fix);
                    if (!FX) break;
                    SN_STAT(2, 1);
                    const bool far = fix && kt >= 0 && kt != prev;
                    if (LZH_SN_AMASK) {
                        const uint64_t KN = ballot(kt < 0);
                        Am = (Am & ~FX) | (FX & ((KN & OKM) | (~KN & OKP)));
                    }
                    if (fix) {
                        ak = kt;
                        oke = kt < 0 ? ok : okp;
                        ce = kt < 0 ? cand : (uint32_t)(base + kt);
                        le = kt < 0 ? len : lep;
                    }
                    const uint64_t FR = ballot(far);
                    if (FR) {                                            // an older member than prev
                        const int k = far ? kt : lane;
                        const uint32_t gw = lane_gather(ps.w, k);
                        const int lf = match_after4(ps, lane_gather(ps.q1, k), lane_gather(ps.q2, k),
                                                    lane_gather(ps.q3, k), lane_gather(ps.q4, k), lane_gather(ps.q5, k));
                        if (far) { le = lf; oke = gw == ps.w; }
                        if (LZH_SN_AMASK) Am = (Am & ~FR) | (FR & ballot(gw == ps.w));
                    }
                }
                SN_CLK(4);
                // ---- records (literal from the previous copy's end, or next_emit)
                if (Mm) {
                    SN_STAT(3, __builtin_popcountll(Mm));
                    const bool mem = lane_on(Mm);
                    int anc;
                    if (LZH_SN_DPPEND) {   // the previous member's end: the running max one lane down
                        const int ep = wave_shr1(ejm);
                        anc = ep > 0 ? base + ep : next_emit;
                    } else {
                    const uint64_t mb = Mm & below;
                    const int jp = mb ? 63 - __builtin_clzll(mb) : lane;
                    const int ep = (int)lane_gather((uint32_t)e, jp);
                    anc = mb ? base + ep : next_emit;
                    }
                    const int lit = p - anc, mlen = 4 + cn;
                    const uint32_t offv = (uint32_t)(p - (int)ce);
                    rc_anc = (uint32_t)anc;
                    rc_lit = kRec ? (uint32_t)(fbase + p) : (uint32_t)lit;   // kRec: the copy start P
                    rc_off = offv;
                    rc_ml = (uint32_t)mlen;
                    rc_m = Mm;
                    if (!kRec) {   // output offsets: only the in-kernel emission needs them
                        int L = 0;
                        if (mem) { const SnapSeq Q(lit, offv, mlen); L = Q.total; }
                        int incl = L;
                        incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xf, 0xf, false);
                        incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xf, 0xf, false);
                        incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xf, 0xf, false);
                        incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xf, 0xf, false);
                        incl += __builtin_amdgcn_update_dpp(0, incl, 0x142, 0xa, 0xf, false);
                        incl += __builtin_amdgcn_update_dpp(0, incl, 0x143, 0xc, 0xf, false);
                        rc_st = (uint32_t)(incl - L);
                        rc_tot = rdlanei(incl, 63);
                    }
                    next_emit = base + eL;
                }
                SN_CLK(5);
                if (endp) break;                                         // remainder from next_emit
                // table: the last inserted lane of each slot, or the slot's old value
                if (LZH_SN_RESTORE2 && !losers) {   // every lane owns its slot: inserted keeps p, else old
                    T.put(h, lane_on(I) ? (uint32_t)p : old);
                    wave_lds_fence();
                } else {   // every lane stores its slot's final value, all lanes of a slot agreeing (a run
                    // batch's 64 probes are all valid): no exec-mask juggling around the store
                    const uint64_t gi = grp & I;
                    T.put(h, gi ? (uint32_t)(base + 63 - __builtin_clzll(gi)) : old);
                    wave_lds_fence();
                }
                if (Mm) {
                    if (eL >= LZH_WAVE) {                                // re-test in a later batch
                        rt = base + eL;
                        org = rt + 1;
                        base = rt - 1;
                    } else {                                             // search continues past the batch
                        rt = -1;
                        org = base + eL + 1;
                        base += LZH_WAVE;
                    }
                } else {
                    rt = -1;
                    base += LZH_WAVE;
                }
                SN_CLK(6);
                continue;
            }

            SN_CLK(6);
            // ================= search batch (sparse probes or near ip_limit): the probe plan
            // along the exact schedule, first hit only (v2)
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
            SREC_OUT();
            rc_m = 0;
            rc_tot = 0;
            {
                const int target = min(front + in.sh + kAhead, endX + 256);
                for (int r = 0; r < 4 && R.fill < target; r++) R.refill(in.r, lane);
            }
            wait_vm();
            R.ready = R.fill;
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
            exact = unii(exact) != 0;
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
                wait_vm();
                R.ready = R.fill;
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
            // (uniform: a phi of `found` / `exact` the compiler takes as divergent turns the batch loop's
            // state into VGPR copies read back by readfirstlane at every iteration)
            found = unii(found) != 0; fh = unii(fh);
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
            {
                rc_anc = (uint32_t)next_emit;
                rc_lit = kRec ? (uint32_t)(fbase + P) : (uint32_t)(P - next_emit);
                rc_off = (uint32_t)(P - M);
                rc_ml = (uint32_t)matched;
                rc_st = 0;
                rc_m = 1;
                if (!kRec) rc_tot = SnapSeq(P - next_emit, (uint32_t)(P - M), matched).total;
            }
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
            // back to run batches: re-test batch at rt (lane 0 = rt-1 insert, lane 1 = rt)
            runm = true;
            base = rt - 1;
            org = rt + 1;
            SN_CLK(7);
        }
    }
#ifdef LZH_SN_CLK
    SN_CLK(7);
    if (lane == 0)
        for (int i = 0; i < 8; i++) atomicAdd(&lzh_sn_clk_buf[i], (unsigned long long)snclk[i]);
    if (lane == 0) atomicAdd(&lzh_sn_clk_buf[8], 1ull);
#endif
    SREC_OUT();
    if (kRec) {   // the fragment's last literal run: a literal-only record
        if (next_emit < fn) {
            if (lane == 0) st_b64(recs, 8 * nrec, (uint32_t)(fbase + fn), 0u);
            nrec++;
        }
        return op;
    }
    if (next_emit < fn) op = emit_seq(in, R, out, op, next_emit, fn - next_emit, 0, 0, lane);
    wave_lds_fence();
    return op;
}

}  // namespace snv2

extern "C" __global__ void __launch_bounds__(64)
lzh_snappy_compress_v2_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                              uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t chunk0,
                              unsigned long long* stats) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[(1 << 13) + 256 + LZH_WAVE / 4];   // table | ring | marks
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
        int nrec = 0;
        op = snv2::compress_fragment<false>(rin, fn, rout, op, (LDSA uint16_t*)lds, (LDSA uint32_t*)lds + (1 << 13),
                                            (LDSA uint8_t*)((LDSA uint32_t*)lds + (1 << 13) + 256), stats,
                                            make_rsrc(nullptr, 0), nrec, 0);
    }
    if (lane == 0) csizes[chunk] = (uint32_t)op;
}

// ======================================================================= parse + emit split
// As for LZ4 (lz4c_hip.hip): the parse kernel (the loop above with kRec, no output marks) leaves
// 8-byte records; lzh_snappy_emit_kernel (no hash table: high occupancy) writes the varint header
// (snappy.cc:1047-1050) and lays out EmitLiteral / EmitCopy (:342-443) for 64 records at a time.

// Records of fragment f of a chunk with more than one fragment start at record f * kFragRecs of the
// chunk's record slot (a 64 KiB fragment has at most 16 384 copies of >= 4 bytes and one closing
// literal-only record), so every fragment is parsed by a wave of its own: snappy starts each
// fragment with a fresh table (snappy.cc:1042-1072), and 64 KiB units balance the CUs better than
// whole chunks at -b256 and above.
constexpr int kFragRecs = 16384 + 32;

extern "C" __global__ void __launch_bounds__(64)
lzh_snappy_parse_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                        uint8_t* recs, uint64_t rec_stride, uint32_t* rec_hdr, uint32_t frags) {
    // (LZH_SN_PADLDS: extra bytes of LDS per wave -- an occupancy experiment, 0 in builds)
    __shared__ __attribute__((aligned(16))) uint32_t lds[(1 << 13) + 256 + 8 + LZH_SN_PADLDS / 4];   // table | ring + mirror
    const uint64_t chunk = blockIdx.x / frags;
    const uint32_t f = blockIdx.x - (uint32_t)chunk * frags;
    const uint64_t off = chunk * chunk_size;
    if (off >= n_total && !(n_total == 0 && chunk == 0)) return;
    const uint32_t n = (uint32_t)min(chunk_size, n_total - off);
    const rsrc_t rr = make_rsrc(recs + chunk * rec_stride, (uint32_t)rec_stride);
    uint32_t* hdr = rec_hdr + chunk * frags;       // end record (exclusive) of each fragment
    int nrec = frags > 1 ? (int)f * kFragRecs : 0;
    const uint32_t fpos = f << 16;
    if (fpos < n) {
        const int fn = (int)min(65536u, n - fpos);
        const uint64_t readable = min<uint64_t>(in_readable - off - fpos, (uint64_t)fn + 64);
        Bytes rin, rout;
        rin.init(in + off + fpos, readable);
        rout.init(nullptr, 0);
        snv2::compress_fragment<true>(rin, fn, rout, 0, (LDSA uint16_t*)lds, (LDSA uint32_t*)lds + (1 << 13), nullptr,
                                      nullptr, rr, nrec, (int)fpos);
    }
    if (threadIdx.x == 0) hdr[f] = (uint32_t)nrec;
}



namespace sne {

#ifndef LZH_SNE_RING
#define LZH_SNE_RING 2048
#endif
constexpr int kRingB = LZH_SNE_RING;    // LDS output ring (bytes)
constexpr int kSpan = LZH_SNE_RING;     // LDS copy of a record group's input span (bytes)

__device__ __forceinline__ int wave_max(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}
__device__ __forceinline__ int wave_excl_scan(int x, int& total) {
    int incl = x;
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x111, 0xf, 0xf, false);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x112, 0xf, 0xf, false);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x114, 0xf, 0xf, false);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x118, 0xf, 0xf, false);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x142, 0xa, 0xf, false);
    incl += __builtin_amdgcn_update_dpp(0, incl, 0x143, 0xc, 0xf, false);
    total = __builtin_amdgcn_readlane(incl, 63);
    return incl - x;
}

// Output ring of one wave writing the byte range [start, end) of a staging slot.  kEdge: other
// waves share the slot (one 64 KiB fragment each) -- dword stores inside the range, byte stores for
// the partial dwords at its edges, so no store touches another wave's bytes; otherwise the range
// starts at 0 and the last partial dword is stored whole.
template <bool kEdge>
struct OutR {
    LDSA uint8_t* b;
    rsrc_t o;          // staging slot (256-aligned)
    int flushed;       // bytes [start, flushed) are in global memory
    __device__ __forceinline__ void put(int pos, uint32_t v) const { ((volatile LDSA uint8_t*)b)[pos & (kRingB - 1)] = (uint8_t)v; }
    __device__ __forceinline__ uint32_t rbyte(int pos) const { return ((volatile LDSA uint8_t*)b)[pos & (kRingB - 1)]; }
    // global <- [flushed, upto): bytes up to the first dword boundary, whole dwords, and (fin) the
    // bytes of the last partial dword; without fin the partial last dword waits for more bytes
    __device__ __forceinline__ void flush(int upto, bool fin, int lane) {
        wave_lds_fence();
        if (!kEdge) {
            const int d0 = flushed >> 2, d1 = fin ? (upto + 3) >> 2 : upto >> 2;
            for (int d = d0 + lane; d < d1; d += 64)
                st_b32(o, 4 * d, ((volatile LDSA uint32_t*)b)[d & (kRingB / 4 - 1)]);
            flushed = 4 * d1;
            if (flushed > upto) flushed = upto & ~3;   // (the partial dword is rewritten by the next flush)
            wave_lds_fence();
            return;
        }
        const int a = flushed, a4 = (a + 3) & ~3, b4 = upto & ~3;
        const int h1 = min(a4, upto);
        if (lane < h1 - a) st_u8(o, a + lane, rbyte(a + lane));
        for (int d = (a4 >> 2) + lane; d < (b4 >> 2); d += 64)
            st_b32(o, 4 * d, ((volatile LDSA uint32_t*)b)[d & (kRingB / 4 - 1)]);
        if (fin) {
            const int t0 = max(a4, b4);
            if (lane < upto - t0) st_u8(o, t0 + lane, rbyte(t0 + lane));
            flushed = upto;
        } else {
            flushed = max(h1, b4);
        }
        wave_lds_fence();
    }
};

constexpr int kBulk = 256;   // literal runs at least this long go straight to HBM (bulk_literals)
// longest literal run the lane-parallel group layout takes (<= 256: a tag and one length byte)
#ifndef LZH_SNE_LITMAX
#define LZH_SNE_LITMAX 256
#endif

}  // namespace sne

namespace sne {

// output bytes of the records [r0, r1) (the first literal run starts at ia)
__device__ int frag_bytes(rsrc_t rr, int r0, int r1, int ia, int lane) {
    int total = 0;
    for (int g = r0; g < r1; g += 64) {
        const int r = g + lane;
        const bool v = r < r1;
        uint32_t w0 = 0, w1 = 0;
        if (v) { w0 = ld_b32(rr, 8 * r); w1 = ld_b32(rr, 8 * r + 4); }
        const int Pc = (int)(w0 & 0xFFFFFFu);
        const int ml = v ? (int)((w0 >> 24) | ((w1 & 0xFFFFu) << 8)) : 0;
        const int end = Pc + ml;
        const int anc = __builtin_amdgcn_update_dpp(ia, end, 0x138, 0xf, 0xf, false);   // wave_shr:1
        const int lit = v ? Pc - anc : 0;
        const snv2::SnapSeq Q(lit, w1 >> 16, ml);
        int T;
        wave_excl_scan(v ? Q.total : 0, T);
        total += T;
        ia = rdlanei(end, min(64, r1 - g) - 1);
    }
    return total;
}

// lay out the records [r0, r1) at op (the first literal run starts at ia); returns the end
// One group of 64 records (lzh_snappy_emit_kernel's pipeline): header from the records (the literal
// run of a record starts at the previous record's end: lane-1 by a wave shift, the previous group's
// end for lane 0) and its input span's dwords, loaded unconditionally into the caller's registers
// (unneeded lanes re-read the span's first dword): a load under a branch merges with the old register
// value, and that copy would wait for the load.
constexpr int kSpanW = kSpan / 256;
struct SGrp {
    int Pc = 0, ml = 0, anc = 0, lit = 0, ia = 0, Lt = 0, X0 = 0, nd = 0;
    uint32_t o = 0;
    bool v = false, span = false;
    __device__ __forceinline__ void head(uint32_t w0, uint32_t w1, int ia_, int g, int r1, const Bytes& in, int lane) {
        v = g + lane < r1;
        Pc = (int)(w0 & 0xFFFFFFu);
        ml = v ? (int)((w0 >> 24) | ((w1 & 0xFFFFu) << 8)) : 0;
        o = w1 >> 16;
        const int end = Pc + ml;
        ia = ia_;
        anc = __builtin_amdgcn_update_dpp(ia_, end, 0x138, 0xf, 0xf, false);   // wave_shr:1
        lit = v ? Pc - anc : 0;
        Lt = __builtin_amdgcn_readlane(end, max(min(64, r1 - g), 1) - 1) - ia_;
        span = Lt + 8 <= kSpan;
        X0 = (ia_ + in.sh) & ~3;
        nd = (ia_ + in.sh + Lt - X0 + 3) >> 2;
    }
    __device__ __forceinline__ void issue(const Bytes& in, int lane, uint32_t* sp) const {
        const int a0 = X0 + 4 * lane;
#pragma unroll
        for (int k = 0; k < kSpanW; k++) sp[k] = ld_b32(in.r, span && 64 * k < nd ? a0 + 256 * k : a0);
    }
};

template <class OutR>
__device__ __forceinline__ int emit_records(OutR& R, const Bytes& in_b, rsrc_t rr, int r0, int r1, int ia, int op,
                            LDSA uint32_t* ibuf, int lane) {
    // Software pipeline over groups of 64 records (as lzh_lz4_emit_kernel): while group g is laid
    // out, group g+1's input span and the records of group g+2 are in flight.
    SGrp GA, GB;                                  // headers of groups g and g+1 (alternating roles)
    uint32_t sp[kSpanW];                          // group g's span dwords (in flight)
    // records of group g+1 (in flight); offsets past the chunk's records are out of range (0)
    uint32_t nw0 = ld_b32(rr, 8 * (r0 + 64 + lane)), nw1 = ld_b32(rr, 8 * (r0 + 64 + lane) + 4);
    {
        const uint32_t w0 = ld_b32(rr, 8 * (r0 + lane)), w1 = ld_b32(rr, 8 * (r0 + lane) + 4);
        GA.head(w0, w1, ia, r0, r1, in_b, lane);
        GA.issue(in_b, lane, sp);
    }
    auto step = [&](SGrp& G, SGrp& Gn, int g) {
        if (G.span) {   // group g's input span [ia, ia + Lt) into LDS (literal bytes are read from there)
#pragma unroll
            for (int k = 0; k < kSpanW; k++)
                if (64 * k < G.nd && lane + 64 * k < G.nd) ibuf[lane + 64 * k] = sp[k];
            wave_lds_fence();
        }
        {   // group g+1: header from its records; its span and the records of group g+2 go out now
            const uint32_t w0 = nw0, w1 = nw1;
            nw0 = ld_b32(rr, 8 * (g + 128 + lane));
            nw1 = ld_b32(rr, 8 * (g + 128 + lane) + 4);
            Gn.head(w0, w1, G.ia + G.Lt, g + 64, r1, in_b, lane);
            Gn.issue(in_b, lane, sp);
        }
        const bool v = G.v;
        const int ml = G.ml, anc = G.anc, lit = G.lit, X0 = G.X0;
        const uint32_t o = G.o;
        const snv2::SnapSeq Q(lit, o, ml);
        const int S = v ? Q.total : 0;
        int T;
        const int pos = op + sne::wave_excl_scan(S, T);
        const int litmax = (int)uni((uint32_t)sne::wave_max(lit));
        if (T <= sne::kRingB / 2 && litmax <= LZH_SNE_LITMAX && G.span) {
            const LDSA uint8_t* ib = (const LDSA uint8_t*)ibuf;
            const int ioff = in_b.sh - X0;            // input position p lives at ib[p + ioff]
            if (op + T - R.flushed > sne::kRingB - 8) R.flush(op, false, lane);
            // every lane writes its own (literal, copy) pair phase by phase (snappy.cc:342-443):
            // tag and (lit <= 64 here) at most one length byte, the literal run (a lane-parallel
            // copy as long as the group's longest), the 64 / 60-byte COPY_2 pieces of a long copy,
            // the final COPY_1 or COPY_2
            if (v && lit > 0) {
                R.put(pos, Q.tag);
                if (Q.hl > 1) R.put(pos + 1, Q.nm1 & 0xffu);
            }
            for (int t = 0; t < litmax; t++)
                if (t < lit) R.put(pos + Q.lit0 + t, ib[anc + t + ioff]);
            const int cp = pos + Q.lit1;
            const int np = v && ml > 0 ? Q.k + Q.has60 : 0;
            for (int i = 0; ballot(i < np); i++) {
                if (i < np) {
                    R.put(cp + 3 * i, i < Q.k ? (2u | (63u << 2)) : (2u | (59u << 2)));
                    R.put(cp + 3 * i + 1, Q.lo);
                    R.put(cp + 3 * i + 2, Q.hi);
                }
            }
            if (v && ml > 0) {
                const int fp = cp + Q.pre;
                if (Q.c1) {
                    R.put(fp, 1u | ((uint32_t)(Q.rem - 4) << 2) | ((Q.offv >> 8) << 5));
                    R.put(fp + 1, Q.lo);
                } else {
                    R.put(fp, 2u | ((uint32_t)(Q.rem - 1) << 2));
                    R.put(fp + 1, Q.lo);
                    R.put(fp + 2, Q.hi);
                }
            }
            op += T;
            if (op - R.flushed >= sne::kRingB / 2) R.flush(op, false, lane);
            wave_lds_fence();
        } else {
            for (int k = 0; k < 64 && g + k < r1; k++) {
                const int kl = rdlanei(lit, k), km = rdlanei(ml, k), ka = rdlanei(anc, k);
                const uint32_t ko = rdlane(o, k);
                const snv2::SnapSeq K(kl, ko, km);
                int t0 = 0;
                if (kl >= sne::kBulk) {   // long literal run: header through the ring, body straight to HBM
                    if (op + 64 - R.flushed > sne::kRingB) R.flush(op, false, lane);
                    if (lane < K.lit0) R.put(op + lane, K.byte(lane, 0u));
                    bulk_literals<sne::kRingB>(R, in_b, ka, op + K.lit0, kl, lane);
                    t0 = K.lit1;
                }
                for (int b = t0; b < K.total; b += 64) {
                    if (op + b + 64 - R.flushed > sne::kRingB) R.flush(op + b, false, lane);
                    const int t = b + lane;
                    const int li = t - K.lit0;
                    const uint32_t lb = (li >= 0 && li < kl) ? in_b.b(ka + li) : 0u;
                    if (t < K.total) R.put(op + t, K.byte(t, lb));
                }
                op += K.total;
            }
        }
    };
    for (int g = r0; g < r1; g += 128) {
        step(GA, GB, g);
        if (g + 64 < r1) step(GB, GA, g + 64);
    }
    return op;
}

}  // namespace sne

// One workgroup per chunk, one wave per 64 KiB fragment (W waves, looping when a chunk has more
// fragments): each wave sums its fragment's output bytes from the records, the fragments' offsets
// follow by a prefix over them, and each wave lays its fragment out at its offset.  (-b64: one
// wave per chunk; -b256: four, where one wave per chunk left half the wave slots idle.)
namespace sne {
constexpr int kSpanDw = kSpan / 4 + 4;   // LDS dwords of a wave's input span
constexpr int kMaxFrags = 256;           // 16 MiB chunks (the split path's limit)

// (the rings, spans and sizes are separate __shared__ arrays: through one shared base the compiler
// cannot tell the span reads from the ring writes apart and serialises the literal copy)
template <bool kMulti>
__device__ __forceinline__ void emit_chunk(LDSA uint8_t* rings, LDSA uint32_t* ibufs, LDSA uint32_t* fsz,
                                           const uint8_t* in, uint64_t n_total, uint64_t in_readable,
                                           uint64_t chunk_size, const uint8_t* recs, uint64_t rec_stride,
                                           const uint32_t* rec_hdr, uint8_t* stage, uint64_t stride, uint32_t* csizes,
                                           uint32_t frags) {
    const int lane = threadIdx.x & 63, wave = kMulti ? threadIdx.x >> 6 : 0, W = kMulti ? blockDim.x >> 6 : 1;
    const uint64_t chunk = blockIdx.x;
    const uint64_t off = chunk * chunk_size;
    if (off >= n_total && !(n_total == 0 && chunk == 0)) return;
    const uint32_t n = (uint32_t)min(chunk_size, n_total - off);
    LDSA uint8_t* ring = rings + wave * kRingB;
    LDSA uint32_t* ibuf = ibufs + wave * kSpanDw;
    Bytes in_b;
    in_b.init(in + off, min<uint64_t>(in_readable - off, (uint64_t)n + 64));
    const rsrc_t rr = make_rsrc(recs + chunk * rec_stride, (uint32_t)rec_stride);
    const uint32_t* hdr = rec_hdr + chunk * frags;
    const int nf = (int)((n + 65535u) >> 16);
    const rsrc_t so = make_rsrc(stage + chunk * stride, (uint32_t)stride);
    int nb = 1;                                    // varint32 uncompressed length (snappy.cc:1047-1050)
    for (uint32_t v = n; v >= 128; v >>= 7) nb++;
    if constexpr (!kMulti) {   // one fragment (chunks of at most 64 KiB)
        OutR<false> R{ring, so, 0};
        if (lane < nb) R.put(lane, ((n >> (7 * lane)) & 0x7fu) | (lane + 1 < nb ? 0x80u : 0u));
        const int e = emit_records(R, in_b, rr, 0, (int)uni(hdr[0]), 0, nb, ibuf, lane);
        R.flush(e, true, lane);
        if (lane == 0) csizes[chunk] = (uint32_t)e;
    } else {
    // sizes of all fragments but the last (the last one's end is the chunk's compressed size)
    for (int f = wave; f < nf - 1; f += W) {
        const int r0 = f * kFragRecs, r1 = (int)uni(hdr[f]);
        const int bytes = frag_bytes(rr, r0, r1, f << 16, lane);
        if (lane == 0) fsz[f] = (uint32_t)bytes;
    }
    if (kMulti) __syncthreads();
    // the varint goes through fragment 0's ring (an empty chunk: a store of its own)
    const uint32_t vb = ((n >> (7 * lane)) & 0x7fu) | (lane + 1 < nb ? 0x80u : 0u);
    if (nf == 0 && wave == 0) {
        if (lane < nb) st_u8(so, lane, vb);
        if (lane == 0) csizes[chunk] = (uint32_t)nb;
    }
    int base = nb;
    for (int f = 0; f < nf; f++) {
        if ((f % W) == wave) {
            const int r0 = f * kFragRecs, r1 = (int)uni(hdr[f]);
            OutR<kMulti> R{ring, so, f == 0 ? 0 : base};
            if (f == 0 && lane < nb) R.put(lane, vb);
            const int e = emit_records(R, in_b, rr, r0, r1, f << 16, base, ibuf, lane);
            R.flush(e, true, lane);
            if (f == nf - 1 && lane == 0) csizes[chunk] = (uint32_t)e;
        }
        if (f < nf - 1) base += (int)uni(((volatile LDSA uint32_t*)fsz)[f]);
    }
    }
}

}  // namespace sne

// -b64 and smaller chunks: a single fragment, one wave
extern "C" __global__ void __launch_bounds__(64)
lzh_snappy_emit_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                       const uint8_t* recs, uint64_t rec_stride, const uint32_t* rec_hdr, uint8_t* stage,
                       uint64_t stride, uint32_t* csizes, uint32_t frags) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[sne::kRingB];
    __shared__ __attribute__((aligned(16))) uint32_t ibuf[sne::kSpanDw];
    sne::emit_chunk<false>((LDSA uint8_t*)ring, (LDSA uint32_t*)ibuf, nullptr, in, n_total, in_readable, chunk_size,
                           recs, rec_stride, rec_hdr, stage, stride, csizes, frags);
}

// larger chunks: kW >= min(fragments, 8) waves (the block has exactly that many), each with its
// ring and span, and the fragment sizes
template <int kW>
__global__ void __launch_bounds__(64 * kW)
lzh_snappy_emit_frag_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                            const uint8_t* recs, uint64_t rec_stride, const uint32_t* rec_hdr, uint8_t* stage,
                            uint64_t stride, uint32_t* csizes, uint32_t frags) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[kW * sne::kRingB];
    __shared__ __attribute__((aligned(16))) uint32_t ibuf[kW * sne::kSpanDw];
    __shared__ uint32_t fsz[sne::kMaxFrags];
    sne::emit_chunk<true>((LDSA uint8_t*)ring, (LDSA uint32_t*)ibuf, (LDSA uint32_t*)fsz, in, n_total, in_readable,
                          chunk_size, recs, rec_stride, rec_hdr, stage, stride, csizes, frags);
}

#include "launch.h"
uint32_t lzh_snappy_frags(uint64_t chunk_size) { return (uint32_t)((chunk_size + 65535) >> 16); }
size_t lzh_snappy_rec_stride(uint64_t chunk_size) {
    const uint32_t frags = lzh_snappy_frags(chunk_size);
    if (frags > 1) return (size_t)frags * kFragRecs * 8;   // (kFragRecs * 8 is a multiple of 256)
    return ((chunk_size / 4 + 8) * 8 + 255) / 256 * 256;
}

// parse kernel + emit kernel (records: nchunks x rec_stride bytes, then a u32 count per chunk);
// stage_mask bit 0 = parse, bit 1 = emit
hipError_t lzh_launch_snappy_split(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                   uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks, uint8_t* recs,
                                   int stage_mask, hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    const uint64_t rs = lzh_snappy_rec_stride(chunk_size);
    uint32_t* hdr = (uint32_t*)(recs + rs * nchunks);
    const uint32_t frags = lzh_snappy_frags(chunk_size);
    if (stage_mask & 1)
        hipLaunchKernelGGL(lzh_snappy_parse_kernel, dim3(nchunks * frags), dim3(64), 0, s, in, n_total, in_readable,
                           chunk_size, recs, rs, hdr, frags);
    if (stage_mask & 2) {
        if (frags > (uint32_t)sne::kMaxFrags) return hipErrorInvalidValue;
        const uint32_t W = frags < 8 ? frags : 8;
#define LZH_SNE_ARGS in, n_total, in_readable, chunk_size, (const uint8_t*)recs, rs, (const uint32_t*)hdr, stage, stride, csizes, frags
        if (W <= 1)
            hipLaunchKernelGGL(lzh_snappy_emit_kernel, dim3(nchunks), dim3(64), 0, s, LZH_SNE_ARGS);
        else if (W == 2)
            hipLaunchKernelGGL(lzh_snappy_emit_frag_kernel<2>, dim3(nchunks), dim3(128), 0, s, LZH_SNE_ARGS);
        else if (W <= 4)
            hipLaunchKernelGGL(lzh_snappy_emit_frag_kernel<4>, dim3(nchunks), dim3(64 * W), 0, s, LZH_SNE_ARGS);
        else
            hipLaunchKernelGGL(lzh_snappy_emit_frag_kernel<8>, dim3(nchunks), dim3(64 * W), 0, s, LZH_SNE_ARGS);
#undef LZH_SNE_ARGS
    }
    return hipGetLastError();
}

hipError_t lzh_launch_snappy_compress_v2(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                         uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks,
                                         hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(lzh_snappy_compress_v2_kernel, dim3(nchunks), dim3(64), 0, s, in, n_total, in_readable,
                       chunk_size, stage, stride, csizes, 0u, (unsigned long long*)nullptr);
    return hipGetLastError();
}

#ifdef LZH_SN_CLK
extern "C" int lzh_debug_snappy_clocks(unsigned long long* host, int reset) {
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(snv2::lzh_sn_clk_buf), 16 * sizeof(unsigned long long)) != hipSuccess) return -1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(snv2::lzh_sn_clk_buf), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif
