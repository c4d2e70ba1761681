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
// (counted per wave in registers, flushed once at the end: per-event atomics would serialize the run)
#define LZ_STAT(i, v) do { if (kStats) ctr[i] += (uint32_t)(v); } while (0)
constexpr int kCtr = 13;
// phase clocks (stats build only): time since the previous mark is charged to phase i
#ifdef LZH_ISA_MARKS   // phase markers in the ISA (tools: instruction counts per phase); off in builds
#define LZ_MARK(i) asm volatile("; LZMARK " #i ::: "memory")
#else
#define LZ_MARK(i) ((void)0)
#endif
#define LZ_CLK(i) do { if (!kStats) LZ_MARK(i); if (kStats) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); clk[i] += t_ - clk_last; clk_last = t_; } } while (0)
constexpr int kClk = 12;

constexpr int kMinMatch = 4;
constexpr int kMfLimit = 12;
constexpr int kLastLiterals = 5;
constexpr int kMinLength = 13;
constexpr int kRing = 1024;           // bytes of LDS input ring per wave
constexpr int kAhead = 704;           // keep the ring filled this far past the batch front
constexpr int kOut = 512;             // bytes of LDS output ring per wave

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
// Refills are LDS-DMA (buffer_load ... lds) issued after a batch's load wait, so they complete
// under the next batch: `ready` is the fill level known to have landed (set at each wait).
struct Ring {
    LDSA uint32_t* w;
    int sh;
    int fill;
    int ready;
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

__device__ __forceinline__ int ext_len_bytes(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

// LDS output ring (kOut bytes) indexed by the output descriptor offset X = pos + sh, so ring
// dwords line up with global dwords: sequences are assembled here with ds_write_b8 and leave
// for HBM as aligned dword stores once 256 bytes are pending (no store in the batch's vmcnt
// wait; one store instruction per 256 output bytes instead of one per sequence).
struct OutRing {
    LDSA uint8_t* b;
    int sh;
    int flushed;          // output bytes [0, flushed) are in global memory
    __device__ __forceinline__ void put(int pos, uint32_t v) const {
        ((volatile LDSA uint8_t*)b)[(pos + sh) & (kOut - 1)] = (uint8_t)v;
    }
    __device__ __forceinline__ uint32_t get(int pos) const {
        return ((volatile const LDSA uint8_t*)b)[(pos + sh) & (kOut - 1)];
    }
    __device__ __forceinline__ uint32_t dword(int X) const {
        return ((volatile const LDSA uint32_t*)b)[(X & (kOut - 1)) >> 2];
    }
    // global <- ring bytes [flushed, upto): aligned dwords, bytewise partial dwords at the ends
    __device__ __forceinline__ void flush(const Bytes& out, int upto, int lane) {
        const int fx = flushed + sh, ux = upto + sh;
        wave_lds_fence();
        for (int D0 = fx & ~3; D0 < ux; D0 += 4 * LZH_WAVE) {
            const int D = D0 + 4 * lane;
            const uint32_t w = dword(D);
            if (D >= fx && D + 4 <= ux) {
                st_b32(out.r, D, w);
            } else if (D + 4 > fx && D < ux) {
#pragma unroll
                for (int k = 0; k < 4; k++)
                    if (D + k >= fx && D + k < ux) st_u8(out.r, D + k, (w >> (8 * k)) & 0xffu);
            }
        }
        flushed = upto;
    }
};

// byte t of a sequence (token, literal-length bytes, literals, offset, match-length bytes)
struct SeqLayout {
    int lx, mx, lit0, lit1, total;
    uint32_t token, lrem, mrem;
    __device__ __forceinline__ SeqLayout(int lit, bool has_match, int ml) {
        lx = ext_len_bytes(lit);
        mx = has_match ? ext_len_bytes(ml) : 0;
        lit0 = 1 + lx;
        lit1 = lit0 + lit;
        total = lit1 + (has_match ? 2 + mx : 0);
        token = ((uint32_t)min(lit, 15) << 4) | (has_match ? (uint32_t)min(ml, 15) : 0u);
        lrem = (uint32_t)(lit - 15) % 255u;
        mrem = (uint32_t)(ml - 15) % 255u;
    }
    __device__ __forceinline__ uint32_t byte(int t, uint32_t lb, int off) const {
        const int u = t - (lit1 + 2);
        uint32_t v = token;
        v = (t >= 1 && t < lit0) ? (t == lx ? lrem : 255u) : v;
        v = (t >= lit0 && t < lit1) ? lb : v;
        v = t == lit1 ? ((uint32_t)off & 0xffu) : v;
        v = t == lit1 + 1 ? ((uint32_t)off >> 8) : v;
        v = (u >= 0) ? (u == mx - 1 ? mrem : 255u) : v;
        return v;
    }
};

// Emit one sequence (has_match) or the final literal run at op; returns the new op.
// Common case (<= 256 bytes, literals in the input ring): assembled in the output ring.
__device__ __forceinline__ int emit_seq(const Bytes& in, const Ring& R, const Bytes& out, OutRing& O, int op,
                                        int anchor, int lit, bool has_match, int off, int ml, int lane) {
    // (ml counts match bytes beyond the 4-byte minimum, as the token does)
    if (has_match && lit < 15 && ml < 15 && R.has(anchor, anchor + 16)) {
        // short sequence (no length bytes): token, lit literals, 2-byte offset
        const uint32_t lb = R.byte(anchor + lane - 1);
        uint32_t v = ((uint32_t)lit << 4) | (uint32_t)ml;
        v = (lane >= 1 && lane <= lit) ? lb : v;
        v = lane == lit + 1 ? ((uint32_t)off & 0xffu) : v;
        v = lane == lit + 2 ? ((uint32_t)off >> 8) : v;
        if (lane < lit + 3) O.put(op + lane, v);
        op += lit + 3;
        if (op - O.flushed >= 4 * LZH_WAVE) O.flush(out, ((op + O.sh) & ~3) - O.sh, lane);
        return op;
    }
    const SeqLayout S(lit, has_match, ml);
    const bool lit_in_ring = R.has(anchor, anchor + lit);
    if (S.total <= 4 * LZH_WAVE && (lit_in_ring || lit <= 2 * LZH_WAVE)) {
        for (int base = 0; base < S.total; base += LZH_WAVE) {
            const int t = base + lane;
            const int lp = anchor + t - S.lit0;
            uint32_t lb = 0;
            if (lit_in_ring) lb = R.byte(lp);
            else if (t >= S.lit0 && t < S.lit1) lb = in.b(lp);
            if (t < S.total) O.put(op + t, S.byte(t, lb, off));
        }
        op += S.total;
        if (op - O.flushed >= 4 * LZH_WAVE) O.flush(out, ((op + O.sh) & ~3) - O.sh, lane);
        return op;
    }
    // long sequence: drain the ring, then write straight to global memory
    O.flush(out, op, lane);
    if (lane == 0) out.st8(op, S.token);
    for (int b = lane; b < S.lx; b += LZH_WAVE) out.st8(op + 1 + b, b == S.lx - 1 ? S.lrem : 255u);
    if (lit_in_ring) {
        for (int base = 0; base < lit; base += LZH_WAVE)
            if (base + lane < lit) out.st8(op + S.lit0 + base + lane, R.byte(anchor + base + lane));
    } else {
        copy_span(in, anchor, out, op + S.lit0, lit, lane, LZH_WAVE);
    }
    if (has_match) {
        if (lane < 2) out.st8(op + S.lit1 + lane, lane ? ((uint32_t)off >> 8) : ((uint32_t)off & 0xffu));
        for (int b = lane; b < S.mx; b += LZH_WAVE) out.st8(op + S.lit1 + 2 + b, b == S.mx - 1 ? S.mrem : 255u);
    }
    op += S.total;
    O.flushed = op;
    return op;
}

// Wave-wide inclusive prefix sum (DPP row shifts + row broadcasts, no LDS round trip).
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return x;
}

#ifndef LZH_LZ4_DPPEND
#define LZH_LZ4_DPPEND 1
#endif
#ifndef LZH_LZ4_RESTORE2
#define LZH_LZ4_RESTORE2 1
#endif
#ifndef LZH_LZ4_RW   // the parse kernel without its LDS input ring: register-window P sides, 10 waves per CU
#define LZH_LZ4_RW 1
#endif
#ifndef LZH_LZ4_WALK4   // the chain walk with one register (4 instructions a member instead of 6)
#define LZH_LZ4_WALK4 1
#endif
#ifndef LZH_LZ4_MASKS   // the resolve's probed / inserted sets as lane masks (no VGPR round trips)
#define LZH_LZ4_MASKS 1
#endif
#ifndef LZH_LZ4_PADLDS
#define LZH_LZ4_PADLDS 0
#endif
#ifndef LZH_LZ4_EXPECT   // run batches as the likely branch (block frequencies for the register allocator; the run
                         // batch's state updates as selects instead were 1-2 % slower, profiles/r06_o)
#define LZH_LZ4_EXPECT 1
#endif
#define RUNB_LIKELY(x) (LZH_LZ4_EXPECT ? __builtin_expect((x) != 0, 1) : (x) != 0)
#ifndef LZH_LZ4_RUNB_SGPR   // the run / stride flag without a readfirstlane at the batch loop's head
#define LZH_LZ4_RUNB_SGPR 1
#endif
#ifndef LZH_LZ4_SWP   // the switch to stride batches at the next batch's head (not on the run batches' back edge)
#define LZH_LZ4_SWP 1
#endif
#ifndef LZH_LZ4_PRFRESH   // the stride path writes the deferred record fields too (no back-edge VGPR copies)
#define LZH_LZ4_PRFRESH 1
#endif
#ifndef LZH_LZ4_AMASK   // the resolve's hit set A as a uniform mask built from single-compare ballots
#define LZH_LZ4_AMASK 1
#endif

// Sequences found by one batch, one per member lane (the lane of the sequence's match start):
// anchor, literal count, offset, match length - 4, first output byte within the batch's
// output.  Emitted lane-parallel under the NEXT batch's candidate loads.  Plain locals (a
// struct here ends up in scratch memory).
#define RECS_DECL                                                                                  \
    uint32_t rc_anc = 0, rc_lit = 0, rc_off = 0, rc_mlx = 0, rc_st = 0, rc_p = 0;                  \
    uint64_t rc_m = 0;                                                                             \
    int rc_tot = 0
#define RECS_EMIT() op = emit_recs(in, R, out, O, op, rc_anc, rc_lit, rc_off, rc_mlx, rc_st, rc_m, rc_tot, lane)
// kRec: the batch's sequences leave as records (match start P | match length - 4 << 24 | offset << 48,
// one u64 per sequence, chunk order, before catch-up) for lzh_lz4_emit_kernel instead of being
// assembled here; the literal run of a record starts at the previous record's match end
#define RECS_OUT()                                                                                 \
    do {                                                                                           \
        if (kRec) {                                                                                \
            const uint64_t rm_ = uni64(rc_m);   /* (wave-uniform: keep it in SGPRs) */             \
            recs_st = rm_ != 0;                                                                    \
            if (rm_) {                                                                             \
                const int ri_ = nrec + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(rm_ >> 32),       \
                                           __builtin_amdgcn_mbcnt_lo((uint32_t)rm_, 0u));          \
                if (lane_on(rm_))                                                                  \
                    st_b64(recs, 8 * ri_, rc_lit | (rc_mlx << 24), (rc_mlx >> 8) | (rc_off << 16));  \
                nrec = unii(nrec + __builtin_popcountll(rm_));                                     \
            }                                                                                      \
        } else {                                                                                   \
            RECS_CHECK();                                                                          \
            RECS_EMIT();                                                                           \
        }                                                                                          \
    } while (0)
// (kLinked) limitedOutput: the first sequence whose match-length check fails (lz4.c:1097-1121: the
// output after its offset + LASTLITERALS + 1 + its match-length bytes past cap) ends the block
#define RECS_CHECK()                                                                               \
    do {                                                                                           \
        if (kLinked && rc_m) {                                                                     \
            const int lt_ = (int)rc_lit, ml_ = (int)rc_mlx;                                        \
            const bool f_ = lane_on(rc_m) &&                                                       \
                            op + (int)rc_st + 9 + ext_len_bytes(lt_) + lt_ + (ml_ + 240) / 255 > lk->cap; \
            const uint64_t fm_ = ballot(f_);                                                       \
            if (fm_) {                                                                             \
                aborted = true;                /* (ends the batch loop) */                        \
                lk->abort = rdlanei((int)rc_p, __builtin_ctzll(fm_));                              \
                rc_m = 0;                                                                          \
            }                                                                                      \
        }                                                                                          \
    } while (0)

// Emit the records at op (returns the new op).  Common case (<= 256 bytes, literals in the
// input ring): output byte t of the batch is lane t of pass t/64; its sequence is the last
// member whose start is <= t.  Else sequence by sequence.
__device__ __forceinline__ int emit_recs(const Bytes& in, const Ring& R, const Bytes& out, OutRing& O, int op,
                                         uint32_t anc, uint32_t lit, uint32_t off, uint32_t mlx, uint32_t st,
                                         uint64_t mem, int tot, int lane) {
    if (mem == 0) return op;
    const int first = __builtin_ctzll(mem), last = 63 - __builtin_clzll(mem);
    const int a0 = rdlanei((int)anc, first), a1 = rdlanei((int)anc, last) + rdlanei((int)lit, last);
    if (tot <= 4 * LZH_WAVE && R.has(a0, a1)) {
        int carry = first;
        // offset (< 2^16) and output start (< 256 on this path) in one gathered word (packing
        // lit | mlx << 8 as well measured 0.3 % slower)
        const uint32_t os = off | (st << 16);
        for (int pass = 0; pass * LZH_WAVE < tot; pass++) {
            const int ob = pass * LZH_WAVE + lane;
            // owner of output byte ob: the last member starting at or before it.  Start marks go
            // into this pass's own (not yet written) output bytes of the ring: cleared to 0xff,
            // each member writes its lane at its start, every lane reads its byte back.
            O.put(op + ob, 0xffu);
            wave_lds_fence();
            const int stl = (int)st;
            if (lane_on(mem) && stl >= pass * LZH_WAVE && stl < (pass + 1) * LZH_WAVE)
                O.put(op + stl, (uint32_t)lane);
            wave_lds_fence();
            const int mv = (int)O.get(op + ob);
            const uint64_t smask = ballot(mv != 0xff);
            const uint64_t le = smask & ((2ull << lane) - 1ull);
            const int own = (int)lane_gather((uint32_t)mv, le ? 63 - __builtin_clzll(le) : lane);
            const int k = le ? own : carry;
            carry = rdlanei(k, 63);
            const int a = (int)lane_gather(anc, k), l = (int)lane_gather(lit, k);
            const int m = (int)lane_gather(mlx, k);
            int o, t;
            const uint32_t osk = lane_gather(os, k);
            o = (int)(osk & 0xffffu);
            t = ob - (int)(osk >> 16);
            const SeqLayout S(l, true, m);
            const uint32_t lb = R.byte(a + t - S.lit0);
            if (ob < tot) O.put(op + ob, S.byte(t, lb, o));
        }
        return op + tot;      // (flushed by the caller after its load wait: no store in that wait)
    }
    for (uint64_t mm = mem; mm; mm &= mm - 1) {
        const int k = __builtin_ctzll(mm);
        op = emit_seq(in, R, out, O, op, rdlanei((int)anc, k), rdlanei((int)lit, k), true, rdlanei((int)off, k),
                      rdlanei((int)mlx, k), lane);
    }
    return op;
}

// Per-lane match evaluation of probe p against candidate c, from 28 bytes around each:
//   P side  [p-4, p+24) from the input ring (or global memory),
//   M side  [c-4, c+24) loaded speculatively for every lane in one 32-byte window.
// ok  : the 4-byte seed matches (LZ4_read32(match) == LZ4_read32(ip), lz4.c:1005)
// bkr : bytes of backward match p-1.. vs c-1.., capped at 4 (catch-up, lz4.c:1017-1020)
// len : bytes of forward match p+4.. vs c+4.., capped at 20 (LZ4_count, lz4.c:603-626)
struct PSide {
    uint32_t m4, w, q0, q1, q2, q3, q4;       // words at p-4, p, p+4, .., p+20
};

// (a single-base read with ds_read2_b32 pairs for batches whose dwords do not wrap was
// measured 1% slower: fewer VALU instructions are not what bounds this kernel)
__device__ __forceinline__ PSide p_side_ring(const Ring& R, int p) {
    const int X = p - 4 + R.sh, A = X & ~3;
    const uint32_t s = (uint32_t)X & 3u;
    const uint32_t a0 = R.dword(A), a1 = R.dword(A + 4), a2 = R.dword(A + 8), a3 = R.dword(A + 12),
                   a4 = R.dword(A + 16), a5 = R.dword(A + 20), a6 = R.dword(A + 24), a7 = R.dword(A + 28);
    PSide v;
    v.m4 = __builtin_amdgcn_alignbyte(a1, a0, s);
    v.w = __builtin_amdgcn_alignbyte(a2, a1, s);
    v.q0 = __builtin_amdgcn_alignbyte(a3, a2, s);
    v.q1 = __builtin_amdgcn_alignbyte(a4, a3, s);
    v.q2 = __builtin_amdgcn_alignbyte(a5, a4, s);
    v.q3 = __builtin_amdgcn_alignbyte(a6, a5, s);
    v.q4 = __builtin_amdgcn_alignbyte(a7, a6, s);
    return v;
}

// the same from a mirrored ring: one base address, immediate offsets, no wrap (kM4: the word at
// p-4, needed only for an in-kernel catch-up)
template <bool kM4>
__device__ __forceinline__ PSide p_side_ring_m(const Ring& R, int p) {
    const int X = p - 4 + R.sh;
    const uint32_t s = (uint32_t)X & 3u;
    const volatile LDSA uint32_t* q = (const volatile LDSA uint32_t*)R.w + ((X & (kRing - 1)) >> 2);
    const uint32_t a0 = kM4 ? q[0] : 0u, a1 = q[1], a2 = q[2], a3 = q[3], a4 = q[4], a5 = q[5], a6 = q[6], a7 = q[7];
    PSide v;
    v.m4 = __builtin_amdgcn_alignbyte(a1, a0, s);
    v.w = __builtin_amdgcn_alignbyte(a2, a1, s);
    v.q0 = __builtin_amdgcn_alignbyte(a3, a2, s);
    v.q1 = __builtin_amdgcn_alignbyte(a4, a3, s);
    v.q2 = __builtin_amdgcn_alignbyte(a5, a4, s);
    v.q3 = __builtin_amdgcn_alignbyte(a6, a5, s);
    v.q4 = __builtin_amdgcn_alignbyte(a7, a6, s);
    return v;
}

__device__ __forceinline__ PSide p_side_global(const Bytes& in, int p) {
    const int X = p - 4 + in.sh, A = X & ~3;
    const uint32_t s = (uint32_t)X & 3u;
    // a0 (bytes A..A+3) matters only when A >= 0; its own clamped offset keeps it out of the
    // wide load of a1..a7, whose range check would otherwise fail as a whole at A = -4
    const uint32_t a0 = ld_b32(in.r, max(A, 0)), a1 = ld_b32(in.r, A + 4), a2 = ld_b32(in.r, A + 8),
                   a3 = ld_b32(in.r, A + 12), a4 = ld_b32(in.r, A + 16), a5 = ld_b32(in.r, A + 20),
                   a6 = ld_b32(in.r, A + 24), a7 = ld_b32(in.r, A + 28);
    PSide v;
    v.m4 = __builtin_amdgcn_alignbyte(a1, a0, s);
    v.w = __builtin_amdgcn_alignbyte(a2, a1, s);
    v.q0 = __builtin_amdgcn_alignbyte(a3, a2, s);
    v.q1 = __builtin_amdgcn_alignbyte(a4, a3, s);
    v.q2 = __builtin_amdgcn_alignbyte(a5, a4, s);
    v.q3 = __builtin_amdgcn_alignbyte(a6, a5, s);
    v.q4 = __builtin_amdgcn_alignbyte(a7, a6, s);
    return v;
}

// the same from a register window: lane l of Wc holds the dword at window byte 4l; ol = the lane's position's
// byte offset in the window (0 <= ol, (ol & ~3) + 24 < 256): its seven dwords by ds_bpermute (no LDS allocation)
__device__ __forceinline__ PSide p_side_win(uint32_t Wc, int ol) {
    const int a = ol & ~3;
    const uint32_t s = (uint32_t)ol & 3u;
    const uint32_t a1 = lane_gather_b(Wc, a), a2 = lane_gather_b(Wc, a + 4), a3 = lane_gather_b(Wc, a + 8),
                   a4 = lane_gather_b(Wc, a + 12), a5 = lane_gather_b(Wc, a + 16), a6 = lane_gather_b(Wc, a + 20),
                   a7 = lane_gather_b(Wc, a + 24);
    PSide v;
    v.m4 = 0;   // (no in-kernel catch-up on this path)
    v.w = __builtin_amdgcn_alignbyte(a2, a1, s);
    v.q0 = __builtin_amdgcn_alignbyte(a3, a2, s);
    v.q1 = __builtin_amdgcn_alignbyte(a4, a3, s);
    v.q2 = __builtin_amdgcn_alignbyte(a5, a4, s);
    v.q3 = __builtin_amdgcn_alignbyte(a6, a5, s);
    v.q4 = __builtin_amdgcn_alignbyte(a7, a6, s);
    return v;
}

struct MWin {
    uint32_t d0, d1, d2, d3, d4, d5, d6, d7;
    int sm;
    __device__ __forceinline__ void load(const Bytes& in, uint32_t c, bool valid) {
        const int X = (valid ? (int)c : 0) + in.sh;
        const int A = (X & ~3) - 4;
        sm = X & 3;
        {   // (idle lanes load the chunk's first bytes: in range, and their evaluation is masked)
            // d0 (bytes before the candidate) matters only when A >= 0: clamped, separate load
            // (a merged wide load starting at offset -4 would fail its range check as a whole)
            d0 = ld_b32(in.r, max(A, 0)); d1 = ld_b32(in.r, A + 4); d2 = ld_b32(in.r, A + 8); d3 = ld_b32(in.r, A + 12);
            d4 = ld_b32(in.r, A + 16); d5 = ld_b32(in.r, A + 20); d6 = ld_b32(in.r, A + 24); d7 = ld_b32(in.r, A + 28);
        }
    }
};

__device__ __forceinline__ uint32_t byte_ctz(uint32_t x) { return (uint32_t)__builtin_ctz(x) >> 3; }



// returns ok; sets bkr (0..4) and len (0..20)
__device__ __forceinline__ bool eval_lane(const PSide& P, const MWin& W, bool valid, int& bkr, int& len,
                                          bool* eq = nullptr) {
    const uint32_t s = (uint32_t)W.sm;
    const uint32_t mm4 = __builtin_amdgcn_alignbyte(W.d1, W.d0, s);
    const uint32_t mw = __builtin_amdgcn_alignbyte(W.d2, W.d1, s);
    const uint32_t x0 = P.q0 ^ __builtin_amdgcn_alignbyte(W.d3, W.d2, s);
    const uint32_t x1 = P.q1 ^ __builtin_amdgcn_alignbyte(W.d4, W.d3, s);
    const uint32_t x2 = P.q2 ^ __builtin_amdgcn_alignbyte(W.d5, W.d4, s);
    const uint32_t x3 = P.q3 ^ __builtin_amdgcn_alignbyte(W.d6, W.d5, s);
    const uint32_t x4 = P.q4 ^ __builtin_amdgcn_alignbyte(W.d7, W.d6, s);
    const int l = first_diff20(x0, x1, x2, x3, x4);
    len = l;
    const uint32_t y = P.m4 ^ mm4;
    bkr = y ? (int)((uint32_t)__builtin_clz(y) >> 3) : 4;
    if (eq) *eq = mw == P.w;                 // (the bare compare: its ballot is the compare's own mask)
    return valid && mw == P.w;
}

// Finish the match at P (candidate M) from the hit lane's bkr/len: catch-up bounded by the
// anchor and the block start (lz4.c:1017-1020), count bounded by matchlimit (lz4.c:1055-1100);
// runs past the precomputed windows continue lane-parallel from global memory.
// Returns bk; cnt = bytes matched past P+4.
template <bool kStats>
__device__ __forceinline__ int finish_match(const Bytes& in, int P, int M, int bkr, int len, int anchor, int mlimit,
                                            int& cnt_out, int lane, uint32_t* ctr) {
    const int maxb = min(P - anchor, M);
    int bk = min(bkr, maxb);
    if (bkr == 4 && maxb > 4) {
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
    const int a = P + kMinMatch;
    int cnt = len;
    if (len == 20 && a + cnt < mlimit) {
        LZ_STAT(6, 1);
        for (int it = 0; it < (1 << 10) && a + cnt < mlimit; it++) {
            const int o = cnt + 4 * lane;
            const uint32_t x = in.w32(a + o) ^ in.w32(M + kMinMatch + o);
            const uint64_t ne = ballot(x != 0);
            if (ne) {
                const int l = ffs64(ne);
                cnt += 4 * l + (int)byte_ctz(rdlane(x, l));
                break;
            }
            cnt += 4 * LZH_WAVE;
        }
    }
    cnt_out = min(cnt, mlimit - a);
    return bk;
}

// catch-up past the 4-byte window (lz4.c:1017-1020): bytes matched backwards from P / M,
// bounded by the anchor and the block start; lane-parallel compare, 64 bytes per step
__device__ __forceinline__ int slow_catchup(const Bytes& in, int P, int M, int anchor, int lane) {
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
    return P - ip2;
}

// LZ4_count past the 20-byte window (lz4.c:603-626): bytes matched after P+4 / M+4, from 20 on,
// capped at matchlimit; lane-parallel compare, 256 bytes per step
__device__ __forceinline__ int slow_count(const Bytes& in, int P, int M, int mlimit, int lane) {
    const int a = P + kMinMatch;
    int cnt = 20;
    for (int it = 0; it < (1 << 10) && a + cnt < mlimit; it++) {
        const int o = cnt + 4 * lane;
        const uint32_t x = in.w32(a + o) ^ in.w32(M + kMinMatch + o);
        const uint64_t ne = ballot(x != 0);
        if (ne) {
            const int l = ffs64(ne);
            cnt += 4 * l + (int)byte_ctz(rdlane(x, l));
            break;
        }
        cnt += 4 * LZH_WAVE;
    }
    return min(cnt, mlimit - a);
}

__device__ __forceinline__ int ctz64v(uint64_t x) { return x ? __builtin_ctzll(x) : 64; }

__device__ __forceinline__ uint64_t lane_bits(int lo, int hi) {   // bits lo..hi (0 <= lo <= hi <= 63)
    return ((2ull << hi) - 1ull) & (~0ull << lo);                 // 2 << 63 wraps to 0: all ones
}

// Group lanes by table slot (one ballot per slot that has a collision): grp = lanes sharing
// this lane's slot; prev = the closest earlier lane in it (-1 if none).
__device__ __forceinline__ void slot_groups(uint32_t h, bool valid, uint64_t losers, uint64_t& grp, int& prev,
                                            int lane) {
    uint64_t pending = losers;
    grp = 1ull << lane;
    prev = -1;
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
}

// Records of a run batch (anchor, literals, offset, match length, output start per member
// lane), built from the batch's pending resolve state: catch-up bounded by the previous match end
// (lz4.c:1017-1020), lengths, DPP prefix sum of the output sizes.
#define RUN_RECORDS()                                                                              \
    do {                                                                                           \
        if (pr_m) {                                                                                \
            LZ_STAT(3, __builtin_popcountll(pr_m));                                                \
            const uint64_t below_ = (1ull << lane) - 1ull;                                         \
            const int p_ = pr_base + lane;                                                         \
            const bool mem_ = lane_on(pr_m);                                               \
            const uint64_t mb_ = pr_m & below_;                                                    \
            const int jp_ = mb_ ? 63 - __builtin_clzll(mb_) : lane;                                \
            const int ep_ = (int)lane_gather((uint32_t)pr_e, jp_);                                 \
            const int anc_ = mb_ ? pr_base + ep_ : pr_anchor;                                      \
            const int maxb_ = min(p_ - anc_, (int)pr_ce);                                          \
            int bk_ = kRec ? 0 : min(pr_be, maxb_);   /* kRec: catch-up in the emission kernel */  \
            const bool scu_ = !kRec && mem_ && pr_be == 4 && maxb_ > 4;                            \
            for (uint64_t sm_ = ballot(scu_); sm_; sm_ &= sm_ - 1) {                               \
                LZ_STAT(5, 1);                                                                     \
                const int k_ = __builtin_ctzll(sm_);                                               \
                const int b_ = slow_catchup(in, pr_base + k_, rdlanei((int)pr_ce, k_), rdlanei(anc_, k_), lane); \
                bk_ = lane == k_ ? b_ : bk_;                                                       \
            }                                                                                      \
            const int lit_ = p_ - bk_ - anc_, mlx_ = bk_ + pr_cn;                                  \
            rc_anc = (uint32_t)anc_;                                                               \
            rc_p = (uint32_t)p_;                                                                   \
            rc_lit = kRec ? (uint32_t)p_ : (uint32_t)lit_;   /* kRec: the match start P */        \
            rc_off = (uint32_t)(p_ - (int)pr_ce);                                                  \
            rc_mlx = (uint32_t)mlx_;                                                               \
            rc_m = pr_m;                                                                           \
            if (!kRec) {   /* output offsets: only the in-kernel emission needs them */            \
                const int L_ = mem_ ? 3 + lit_ + ext_len_bytes(lit_) + ext_len_bytes(mlx_) : 0;    \
                const int incl_ = wave_incl_scan(L_);                                              \
                rc_st = (uint32_t)(incl_ - L_);                                                    \
                rc_tot = rdlanei(incl_, 63);                                                       \
            }                                                                                      \
            pr_m = 0;                                                                              \
        }                                                                                          \
    } while (0)

// One block of an LZ4 frame with linked blocks (kLinked; lzh_lz4f_linked_kernel): the parse of
// LZ4_compress_fast_continue in prefix mode (lz4.c:1565-1628 -> LZ4_compress_generic with byU32,
// withPrefix64k, noDictIssue, limitedOutput): positions are frame indices, the block is
// [b0, b0 + n), the table persists from block to block, candidates reach back into earlier blocks
// (at most 65535 bytes, the byU32 distance check), the catch-up stops at the frame start
// (lowLimit = source - dictSize).  cap = the limitedOutput budget (block size - 1): the first
// sequence whose match-length check fails (lz4.c:1097-1121; it implies the literal check,
// :1024-1027) ends the parse with abort = its probe position, a failing last-literals check
// (:1207-1216) with abort = -2; else -1.  stop >= 0: a table-only replay that ends right after
// the probe at `stop` (the table as the reference leaves it at an abort: positions past stop are not
// probed, a match ending past it ends the parse).  At every end of the parse the table is left as
// the reference leaves it (the next block starts from it).
struct LinkCtl {
    int b0, cap, stop;
    bool keep_tab;       // the table holds the frame's earlier blocks (else zeroed)
    int abort;           // out: -1 fits, >= 0 probe position of the failing sequence, -2 last literals
};

// kFast (acceleration > 1, lz4.c:958-967): run batches probe a data-independent pattern.  A search
// from a segment origin e (a match end, re-tested, or position 0 at the chunk start) probes
// e+1, e+2, then steps of acc for 64 probes: offsets {0, 1, 2, 2+acc, 2+2acc, ..} from e.  Run
// batches cover the first 64 search probes of each segment (as with acc 1); later probes and the
// chunk tail (where a probe's forwardIp could pass mflimit) go through stride batches.
// kRW (records only): no LDS input ring -- the table alone (16 KiB) leaves room for 10 waves per CU instead of 9 --
// and the run batches' P sides come from a register window of the input (see the loop top)
template <bool kSmall, bool kStats, bool kRec = false, bool kFast = false, bool kLinked = false, bool kRW = false>
__device__ void compress_chunk(const Bytes& in, int n, const Bytes& out, int acc, LDSA uint32_t* tab,
                               LDSA uint32_t* ringw, LDSA uint8_t* outb, uint32_t* out_size,
                               unsigned long long* stats, rsrc_t recs, uint32_t* rec_hdr, LinkCtl* lk = nullptr) {
    static_assert(!kLinked || (!kSmall && !kRec), "linked frames: byU32, in-kernel emission");
    const int b0 = kLinked ? lk->b0 : 0;                  // the block's first position (frame index)
    const int lane = threadIdx.x;
    Table<kSmall> T{tab};
    uint64_t clk[kClk] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t ctr[kCtr] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t clk_last = kStats ? __builtin_amdgcn_s_memtime() : 0;
    if (n <= 0) {
        if (kRec) {
            if (lane == 0) { rec_hdr[0] = 0; rec_hdr[1] = 0; }
            return;
        }
        if (lane == 0) out.st8(0, 0);
        if (lane == 0) *out_size = 1;
        return;
    }
    int nrec = 0;
    bool recs_st = false;     // a record store was issued after this batch's candidate loads
    if (!kLinked || !lk->keep_tab) {
        LDSA uint32_t* t4 = (LDSA uint32_t*)tab;
#pragma unroll
        for (int i = 0; i < 16; i++) lds_zero16(t4 + 4 * (i * LZH_WAVE + lane));
    }
    static_assert(!kRW || kRec, "the register window serves the records-only parse");
    // (without the ring and with every P side from memory -- 10 waves -- 6 % slower, profiles/r05_lnr; kRW keeps
    // the P sides off memory's latency with a register window)
    constexpr bool kRingOn = !kRW;
    Ring R{ringw, in.sh, 0, 0, kRingOn, kRec};   // (the parse kernel's ring carries a 32-byte mirror)
    if (kLinked) R.fill = max(((b0 + in.sh) & ~255) - 256, 0);   // (a block's ring starts just before it)
    OutRing O{outb, out.sh, 0};
    const int endX = b0 + n + in.sh + 8;
    for (int s = 0; s < kRing / 256 && R.fill < endX; s++) R.refill(in.r, lane);
    wait_vm();
    R.ready = R.fill;
    wave_lds_fence();

    int op = 0, anchor = b0;
    bool aborted = false;                    // (kLinked) the limitedOutput budget ran out
    if (kLinked) lk->abort = -1;
    RECS_DECL;                               // sequences waiting to be emitted
    uint64_t pr_m = 0;                       // a run batch whose records are not built yet
    int pr_base = 0, pr_anchor = 0, pr_e = 0, pr_cn = 0, pr_be = 0;
    uint32_t pr_ce = 0;

    if (n >= kMinLength) {
        const int mfl1 = b0 + n - kMfLimit + 1;
        const int mlimit = b0 + n - kLastLiterals;
        // (kLinked replay: positions past `stop` are not probed, a match end past it ends the parse)
        const int stop = kLinked && lk->stop >= 0 ? lk->stop : (1 << 30);
        const int mfe = kLinked ? min(mfl1, stop + 1) : mfl1;
        const int64_t a64 = (int64_t)acc << 6;

        {   // the first position enters the table before the first search (lz4.c:922-923)
            const uint64_t v0 = kRingOn ? ((uint64_t)R.u32(b0) | ((uint64_t)R.byte(b0 + 4) << 32)) : in.w40(b0);
            const uint32_t h0 = hash_of<kSmall>((uint32_t)v0, (uint32_t)(v0 >> 32));
            if (lane == 0) T.put(h0, (uint32_t)b0);
            wave_lds_fence();
        }
        // Parse state.  Run batches (acceleration 1, a search in its first 64 probes): lanes
        // are positions base..base+63; the next probe is q, probes step by 1 up to qlim (the
        // re-test at a match end, then 64 step-1 search probes, lz4.c:955-969 / :1148-1200);
        // pins = a pending ip-2 table fill (lz4.c:1145-1146) sitting at base.  Stride batches
        // (any other schedule): one sequence per batch, the search from s with k0 probes done.
        // (ints: uniform SGPR phis, not lane masks; runb 2 = a run batch's 64 probes found nothing, stride batches
        // from the next batch's head on, LZH_LZ4_SWP)
        int runb = kFast || acc == 1, retest = 0, go = 1;
        const int dlim = kFast ? 2 + 62 * acc : 64;      // last run-batch probe: segment origin + dlim
        int base = b0 + 1, q = b0 + 1, qlim = b0 + dlim, pins = -1;
        int so = b0;                             // segment origin (kFast pattern phase)
        int s = b0 + 1, k0 = 0;
        // probe pattern from a segment origin (bits = offsets): PER = {0, acc, 2acc, ..}, PAT = {0, 1, 2 + PER}
        uint64_t PER = ~0ull, PAT = ~0ull;
        if (kFast) {
            PER = 0;
            for (int o = 0; o < LZH_WAVE; o += acc) PER |= 1ull << o;
            PAT = 3ull | (PER << 2);
        }

        // (kRW) register window over the input, one dword a lane: Wc = the 256 bytes at descriptor offset WX (a
        // multiple of 4), Wn = those at WX + 128.  A run batch at base takes its P sides from Wc when its 64
        // positions' bytes lie in it (0 <= base + sh - WX <= kWinMax), else moves the window up by 128 (Wc = Wn)
        // when that covers it, else reads them from memory and restarts the window at its base (2.8 batches per
        // 64 KiB chunk of text, profiles/r06_e).  Wn is reloaded in every batch (unconditionally, so no register
        // merges with a load in flight), after its candidate loads: their wait -- the compiler's, by register --
        // leaves it in flight, and the next batch's window move waits for it.
        constexpr int kWinMax = 168;           // lane 63's last dword ((o + 63) & ~3) + 24 stays below byte 256
        uint32_t Wc = 0, Wn = 0;
        int WX = 0, wc_ok = 0, wn_ok = 0;
        for (int guard = 0;; guard++) {
            // (the loop-carried parse state is wave-uniform: readfirstlane keeps it in SGPRs, and the
            // exit test on uniform values is a scalar branch, not an exec-mask loop exit)
            go = unii(go);
            if (kLinked) aborted = unii(aborted) != 0;
            if (!go || (kLinked && aborted) || guard >= 4 * n + 64) break;
            // (runb: no readfirstlane -- its phi is uniform from constants under uniform branches, and the
            // readfirstlane kept it in a VGPR: a v_mov + v_readfirstlane a batch)
            if (!LZH_LZ4_RUNB_SGPR) runb = unii(runb);
            retest = unii(retest);
            base = unii(base); q = unii(q); qlim = unii(qlim); pins = unii(pins); s = unii(s); k0 = unii(k0);
            op = unii(op); anchor = unii(anchor); rc_tot = unii(rc_tot); nrec = unii(nrec);
            R.fill = unii(R.fill); R.ready = unii(R.ready); O.flushed = unii(O.flushed);
            so = unii(so);
            LZ_STAT(0, 1);
            if (LZH_LZ4_SWP && runb == 2) {   // a run batch's 64 probes found nothing: stride batches from here
                runb = 0;
                s = so + 1;
                k0 = LZH_WAVE;
                retest = 0;
            }
            if (kFast && runb && base + LZH_WAVE - 1 + acc > mfl1) {
                // near the chunk end a probe's forwardIp may pass mflimit: stride batches take over
                // (the pending ip-2 insert first, then the re-test or the next search probe)
                if (pins >= 0) {
                    uint32_t w, bb = 0;
                    if (R.has(pins - 4, pins + 12)) { w = R.u32(pins); if (!kSmall) bb = R.byte(pins + 4); }
                    else { const uint64_t v = in.w40(pins); w = (uint32_t)v; bb = (uint32_t)(v >> 32); }
                    const uint32_t hp = hash_of<kSmall>(w, bb);
                    if (lane == 0) T.put(hp, (uint32_t)pins);
                    wave_lds_fence();
                }
                const int d = q - so;
                s = so + 1;
                retest = d <= 0 ? 1 : 0;
                k0 = d <= 1 ? 0 : 1 + (d - 2 + acc - 1) / acc;
                runb = 0;
            }
            LZ_CLK(9);                                                 // (loop overhead / uncharged)

            // ---- lanes -> positions
            int p;
            bool valid;
            // (the lane mask and the first position per branch, as uniform values: a ballot of the merged `valid`
            // goes through a VGPR, and lane 0's position of a run batch is its base)
            uint64_t vmask;
            int front;
            if (RUNB_LIKELY(runb)) {
                p = base + lane;
                vmask = ballot(p + 1 <= mfl1);                       // forwardIp <= mflimitPlusOne (lz4.c:969)
                if (kLinked) vmask &= ballot(p <= stop);
                valid = lane_on(vmask);
                front = base;
            } else {
                int64_t pp, nxt;
                if (retest && lane == 0) {
                    pp = s - 1;
                    nxt = s;
                } else {
                    const int k = retest ? lane - 1 : k0 + lane;
                    const int64_t o = k == 0 ? 0 : 1 + step_prefix(a64 + k - 1) - step_prefix(a64);
                    const int64_t st = k == 0 ? 1 : (a64 + k - 1) >> 6;
                    pp = (int64_t)s + o;
                    nxt = pp + st;
                }
                valid = nxt <= mfl1 && (!kLinked || pp <= stop);
                p = valid ? (int)pp : 0;
                vmask = ballot(valid);
                front = rdlanei(p, 0);
            }
            vmask = uni64(vmask); front = unii(front);
            const int pmax = vmask ? rdlanei(p, 63 - __builtin_clzll(vmask)) : front;

            // ---- P-side bytes (ring when it covers the batch), hash, table read / claim / read back
            PSide ps;
            uint32_t b4 = 0;
            if (kRW) {
                WX = unii(WX); wc_ok = unii(wc_ok); wn_ok = unii(wn_ok);
                int o = front + in.sh - WX;
                // 1: Wc, 2: the window moved up 128 (scalar ints and unsigned range tests: no lane-mask booleans)
                const int c1 = runb & wc_ok & (int)((unsigned)o <= (unsigned)kWinMax);
                const int c2 = runb & wn_ok & (int)((unsigned)(o - 128) <= (unsigned)kWinMax);
                const int use = c1 ? 1 : (c2 ? 2 : 0);
                if (use == 2) { Wc = Wn; WX += 128; o -= 128; LZ_STAT(4, 1); }
                if (!use) WX = ((front + in.sh) & ~3) - 128;          // (Wn from here on: the next batch's Wc)
                wc_ok = c1 | c2;
                if (use) {
                    ps = p_side_win(Wc, o + lane);
                } else {
                    LZ_STAT(9, 1);
                    ps = p_side_global(in, p);
                }
            } else if (R.has(front - 4, pmax + 28)) {
                ps = kRec ? p_side_ring_m<false>(R, p) : p_side_ring(R, p);
            } else {
                LZ_STAT(9, 1);
                ps = p_side_global(in, p);
            }
            if (!kSmall) b4 = ps.q0 & 0xffu;
            const uint32_t h = hash_of<kSmall>(ps.w, b4);
            LZ_CLK(0);                                                 // lanes -> positions, P side, hash
            const uint32_t old = T.get(h);
            uint32_t cand = old;
            MWin W;
            W.load(in, cand, valid);                                   // (issued before the claim round trip)
            if (vmask == ~0ull) T.put(h, (uint32_t)p);   // (no exec-mask juggling)
            else if (valid) T.put(h, (uint32_t)p);
            wave_lds_fence();
            const uint32_t back = T.get(h);
            const uint64_t losers = ballot(back != (uint32_t)p) & vmask;   // (one compare: no VGPR round trip)
            LZ_CLK(1);                                                 // table read/claim/read back, loads issued
            // ---- deferred records + emission of the previous batch (under the loads above)
            pr_m = uni64(pr_m); pr_base = unii(pr_base); pr_anchor = unii(pr_anchor);
            RUN_RECORDS();
            RECS_OUT();
            rc_m = 0;
            rc_tot = 0;
            LZ_CLK(2);                                                 // deferred emission
            // run batch: the slot groups and the collider pre-evaluation need no candidate bytes,
            // so they run under the candidate loads (a probe whose slot holds an earlier lane of
            // the batch sees that lane's position if it was inserted, else the slot's old value)
            uint64_t grp = 1ull << lane;
            uint64_t coll = 0;
            int prev = -1;
            const uint64_t below = (1ull << lane) - 1ull;
            bool okp = false;                                      // evaluation against lane prev
            uint64_t OKP = 0;                                      // (as a lane mask)
            int bep = 0, lep = 0;
            if (runb && losers) {
                LZ_STAT(1, 1);
                // slot groups without a loop: every lane of a slot read back the same claim
                // winner W (whichever lane the hardware let win), so equal W <=> same slot;
                // equality of the 6-bit W is bit-sliced over 6 ballots (64 group masks in LDS, each lane ORing
                // its bit into its winner's, measured 2 % slower: conflicting LDS atomics, profiles/r06_g)
                const uint32_t W = back - (uint32_t)base;
                uint32_t ne0 = 0, ne1 = 0;                         // lanes whose winner differs in a bit
#pragma unroll
                for (int b = 0; b < 6; b++) {
                    const uint64_t bm = ballot((W >> b) & 1u);
                    const uint32_t mine = (uint32_t)__builtin_amdgcn_sbfe((int)W, b, 1);   // 0 / ~0
                    ne0 |= (uint32_t)bm ^ mine;
                    ne1 |= (uint32_t)(bm >> 32) ^ mine;
                }
                const uint64_t ne = ((uint64_t)ne1 << 32) | ne0;
                grp = valid ? (~ne & vmask) : (1ull << lane);

                const uint64_t eb = grp & below;
                prev = (valid && eb) ? 63 - __builtin_clzll(eb) : -1;
                coll = ballot(eb != 0ull) & vmask;                 // (= lanes with prev >= 0)
                // a collider's candidate is usually its closest earlier slot member: evaluate
                // that pair once per batch (the per-step test below then only selects)
                const int k = prev >= 0 ? prev : lane;
                const uint32_t gm4 = lane_gather(ps.m4, k), gw = lane_gather(ps.w, k),
                               g0 = lane_gather(ps.q0, k), g1 = lane_gather(ps.q1, k),
                               g2 = lane_gather(ps.q2, k), g3 = lane_gather(ps.q3, k),
                               g4 = lane_gather(ps.q4, k);
                const uint32_t x0 = ps.q0 ^ g0, x1 = ps.q1 ^ g1, x2 = ps.q2 ^ g2, x3 = ps.q3 ^ g3,
                               x4 = ps.q4 ^ g4;
                const int l = first_diff20(x0, x1, x2, x3, x4);
                lep = l;
                const uint32_t y = ps.m4 ^ gm4;
                bep = y ? (int)((uint32_t)__builtin_clz(y) >> 3) : 4;
                okp = valid && gw == ps.w;
                OKP = ballot(gw == ps.w) & vmask;
            }
            if (kRW) {
                // the window's next part, after the candidate loads (no explicit wait: the compiler waits for the
                // candidate data by register, which leaves this load in flight)
                Wn = ld_b32(in.r, WX + 128 + 4 * lane);
                wn_ok = 1;                                             // (for the next batch, restarted or not)
            } else {
                // the candidate loads; a record store issued after them need not be acknowledged
                // (vector memory operations complete in issue order)
                if (kRec && recs_st) wait_vm_but1();
                else wait_vm();
            }
            recs_st = false;
            R.ready = R.fill;
            wave_lds_fence();
            LZ_CLK(3);                                                 // exposed load wait
            // ring refill and output flush after the wait: they complete under the next batch
            {
                const int target = min(front + in.sh + kAhead, endX + 256);
                for (int r = 0; r < 4 && R.fill < target; r++) { R.refill(in.r, lane); LZ_STAT(12, 1); }
            }
            if (!kRec && op - O.flushed >= 4 * LZH_WAVE) O.flush(out, ((op + O.sh) & ~3) - O.sh, lane);
            int bkr, len;
            bool eqw;
            bool ok = eval_lane(ps, W, valid, bkr, len, &eqw);
            if (!kSmall) ok = ok && (cand + 65535u >= (uint32_t)p);
            // (LZH_LZ4_AMASK: `ok` as a lane mask, balloted next to its compares -- an i1 that crosses a block
            // boundary goes through a VGPR to be balloted)
            uint64_t OKM = 0;
            if (LZH_LZ4_AMASK) {
                OKM = ballot(eqw) & vmask;
                if (!kSmall) OKM &= ballot(cand + 65535u >= (uint32_t)p);
            }

            if (RUNB_LIKELY(runb)) {
                // ================= run batch: resolve every sequence that starts in the batch
                // ("colliders" are re-evaluated per step against the in-batch candidate)
                LZ_CLK(4);                                             // eval + slot groups
                // the resolve (a serial chain of dependent scalar / lane reads) issues ahead of the other
                // waves' independent work: s_setprio 1 until the table restore (-0.6 %, profiles/r04_d)
                __builtin_amdgcn_s_setprio(1);
                const int fv = __builtin_popcountll(vmask);           // first lane past mflimit
                const uint64_t I0 = pins >= 0 ? (1ull << (pins - base)) : 0ull;
                const int lo = q - base, hi0 = min(qlim - base, LZH_WAVE - 1);
                // probes of the batch's first segment (lanes lo..hi0; under kFast on the pattern)
                uint64_t P0 = lane_bits(lo, hi0);
                if (kFast) {
                    const int off = so - base;
                    uint64_t Mp;
                    if (off >= 0) {
                        Mp = PAT << off;
                    } else {
                        const int u = -off, t = ((2 - u) % acc + acc) % acc;
                        Mp = (t < LZH_WAVE ? PER << t : 0ull) | (u == 1 ? 1ull : 0ull);
                    }
                    P0 &= Mp;
                }
                // Each lane's candidate: the latest earlier slot member that is inserted when the
                // lane is probed (ak; -1 = the slot's old value).  Assume prev, resolve the batch,
                // check the assumption against the resolved inserted set; repeat with corrected
                // candidates until consistent (each round fixes a prefix of the batch).
                int ak = prev;
                bool oke = prev >= 0 ? okp : ok;
                // (LZH_LZ4_AMASK) the lanes whose candidate matches, carried as a uniform mask: a ballot of the
                // merged bool `oke` costs a VGPR round trip per round, the mask costs three scalar operations
                const uint64_t Am0 = (coll & OKP) | (OKM & ~coll);
                uint64_t Am = Am0;
                uint32_t ce = prev >= 0 ? (uint32_t)(base + prev) : cand;
                int be = prev >= 0 ? bep : bkr, le = prev >= 0 ? lep : len;
                uint64_t Mm = 0, I = I0;                               // member lanes (sequence starts)
                int cn = 0, e = 0;                                     // per lane: match count, end lane
                int eL = 0;                                            // end lane of the last member
                bool endp = false;                                     // the parse ends in this batch
                for (int round = 0; round <= LZH_WAVE; round++) {
                    const uint64_t A = LZH_LZ4_AMASK ? uni64(Am) : ballot(oke);
                    // if lane l starts a sequence: match count, end lane, next hit at or after the end
                    cn = min(le, mlimit - (p + kMinMatch));
                    const bool lng = (LZH_LZ4_AMASK ? lane_on(A) : oke) && le == 20 && p + kMinMatch + 20 < mlimit;
                    e = lane + kMinMatch + cn;
                    int f = ctz64v(e < LZH_WAVE ? (A & (PAT << e)) : 0ull);
                    // chain walk (lz4.c:1142-1200: match end -> re-test -> search from ip+1)
                    Mm = 0;
                    endp = false;
                    uint64_t E;                                        // probed lanes
                    const uint64_t r0 = A & P0;
                    if (!r0) {
                        E = P0;
                        endp = hi0 >= fv;                              // ran past mflimit (lz4.c:969)
                    } else {
                        int sl = __builtin_ctzll(r0);
                        bool endip = false;                            // a match ended past mflimit
                        // link: next member lane, or 0x80 for the rare cases (long match, parse end)
                        const int link = (lng || p + kMinMatch + cn >= mfe) ? 0x80 : f;
                        LZ_CLK(10);                            // (stats: per-lane links)
                        // (links strictly increase, so the walks end)
                        for (;;) {
                            int fs;
                            if (LZH_LZ4_WALK4) {
                                // common case: plain links, one register for the walk (the last member is the
                                // highest bit of Mm afterwards: members increase) -- 4 instructions a member
                                fs = unii(sl);
                                Mm = uni64(Mm);   // (uniform already: readfirstlane keeps every instantiation in SGPRs)
                                do {
                                    asm("s_bitset1_b64 %0, %1" : "+s"(Mm) : "s"(fs));
                                    fs = rdlanei(link, fs);
                                } while (fs < LZH_WAVE);
                                sl = 63 - __builtin_clzll(Mm);
                            } else {
                            for (;;) {                                 // common case: plain links
                                Mm |= 1ull << sl;
                                fs = rdlanei(link, sl);
                                if (fs >= LZH_WAVE) break;
                                sl = fs;
                            }
                            }
                            if (fs != 0x80) break;                     // the chain leaves the batch
                            int es;
                            if (rdlane((uint32_t)lng, sl)) {           // match runs past the window
                                LZ_STAT(6, 1);
                                const int c = slow_count(in, base + sl, rdlanei((int)ce, sl), mlimit, lane);
                                es = sl + kMinMatch + c;
                                cn = lane == sl ? c : cn;
                                e = lane == sl ? es : e;
                                fs = ctz64v(es < LZH_WAVE ? (A & (PAT << es)) : 0ull);
                            } else {
                                es = rdlanei(e, sl);
                            }
                            if (base + es >= mfe) { endip = true; break; }   // lz4.c:1142
                            if (fs >= LZH_WAVE) break;
                            sl = fs;
                        }
                        eL = rdlanei(e, sl);
                        LZ_CLK(11);                            // (stats: the scalar walk)
                        // lanes strictly inside a member's match are not probed; ip-2 is inserted
                        if (!kFast && LZH_LZ4_DPPEND) {
                            // the end of the last member at or before each lane: members' ends increase along
                            // the chain (the next member starts at or after the previous end), so it is the
                            // running max of the members' ends -- DPP, no LDS round trip
                            const bool mem = lane_on(Mm);
                            const int ej = wave_incl_max(mem ? e : 0);
                            if (LZH_LZ4_MASKS) {
                                // (as lane masks: one compare each, the rest scalar -- a ballot of a compound
                                // condition goes through a VGPR and back)
                                const uint64_t inside = ballot(lane < ej) & ~Mm;
                                const uint64_t below_eL = endip && eL < LZH_WAVE ? (1ull << eL) - 1ull : ~0ull;
                                E = (~0ull << lo) & ~inside & below_eL;
                                I = ballot(lane + 2 == ej) & ~Mm;      // lz4.c:1146 (a member's own end is >= lane + 4)
                            } else {
                            const bool inside = !mem && lane < ej;
                            E = ballot(lane >= lo && !inside && (!endip || lane < eL));
                            I = ballot(!mem && lane == ej - 2);        // lz4.c:1146 (a member's own end is >= lane + 4)
                            }
                        } else {
                        const uint64_t mle = Mm & (below | (1ull << lane));
                        const int j = mle ? 63 - __builtin_clzll(mle) : lane;
                        const int ej = (int)lane_gather((uint32_t)e, j);
                        const bool inside = mle && lane > j && lane < ej;
                        bool probed = lane >= lo && !inside;
                        if (kFast)   // before the first member: the first segment's pattern; after a
                            probed = mle ? (lane == j || (lane >= ej && ((PAT >> ((lane - ej) & 63)) & 1ull)))
                                         : lane_on(P0);        // member's end: its pattern
                        E = ballot(probed && (!endip || lane < eL));
                        I = ballot(mle && lane == ej - 2);             // lz4.c:1146
                        }
                        endp = endip || (eL < LZH_WAVE && LZH_WAVE - 1 >= fv);   // or the search ran past mflimit
                    }
                    I = (Mm ? I : 0ull) | I0 | E;                          // (no stale bits from an earlier round)
                    if (!(coll & E)) break;
                    const uint64_t mk = grp & below & I;
                    const int kt = mk ? 63 - __builtin_clzll(mk) : -1;
                    const bool fix = lane_on(E) && kt != ak;
                    const uint64_t FX = ballot(fix);
                    if (!FX) break;
                    LZ_STAT(2, 1);
                    const bool far = fix && kt >= 0 && kt != prev;
                    if (LZH_LZ4_AMASK) {
                        const uint64_t KN = ballot(kt < 0);
                        Am = (Am & ~FX) | (FX & ((KN & OKM) | (~KN & OKP)));
                    }
                    if (fix) {
                        ak = kt;
                        if (!LZH_LZ4_AMASK) oke = kt < 0 ? ok : okp;
                        ce = kt < 0 ? cand : (uint32_t)(base + kt);
                        be = kt < 0 ? bkr : bep;
                        le = kt < 0 ? len : lep;
                    }
                    const uint64_t FR = ballot(far);
                    if (FR) {                                          // an older member than prev
                        const int k = far ? kt : lane;
                        const uint32_t gm4 = lane_gather(ps.m4, k), gw = lane_gather(ps.w, k),
                                       g0 = lane_gather(ps.q0, k), g1 = lane_gather(ps.q1, k),
                                       g2 = lane_gather(ps.q2, k), g3 = lane_gather(ps.q3, k),
                                       g4 = lane_gather(ps.q4, k);
                        if (far) {
                            const uint32_t x0 = ps.q0 ^ g0, x1 = ps.q1 ^ g1, x2 = ps.q2 ^ g2, x3 = ps.q3 ^ g3,
                                           x4 = ps.q4 ^ g4;
                            const int l = first_diff20(x0, x1, x2, x3, x4);
                            le = l;
                            const uint32_t y = ps.m4 ^ gm4;
                            be = y ? (int)((uint32_t)__builtin_clz(y) >> 3) : 4;
                            if (!LZH_LZ4_AMASK) oke = valid && gw == ps.w;
                        }
                        if (LZH_LZ4_AMASK) Am = (Am & ~FR) | (FR & ballot(gw == ps.w) & vmask);
                    }
                }
                LZ_CLK(5);                                             // chain resolve
                // ---- records of the members (emitted under the next batch's loads)
                // the sequences' records are built under the next batch's loads (RUN_RECORDS)
                pr_m = Mm; pr_base = base; pr_anchor = anchor; pr_e = e; pr_cn = cn; pr_be = be; pr_ce = ce;
                LZ_CLK(6);                                             // records
                // (kLinked) the table restore at the end of a block (as in the else branch below)
                auto restore = [&](uint64_t Iw) {
                    const bool inI = lane_on(Iw);
                    if (vmask == ~0ull) {
                        // every lane stores its slot's final value (all lanes of a slot agree):
                        // the slot's last inserted lane, else its old value
                        const uint64_t gi = grp & Iw;
                        T.put(h, gi ? (uint32_t)(base + 63 - __builtin_clzll(gi)) : old);
                    } else if (!losers) {
                        if (valid && !inI) T.put(h, old);
                    } else {
                        const uint64_t gi = grp & Iw;
                        const bool wr = valid && (gi == 0 || (inI && (gi & ~((2ull << lane) - 1ull)) == 0));
                        if (wr) T.put(h, inI ? (uint32_t)p : old);
                    }
                    wave_lds_fence();
                };
                if (endp) {
                    go = 0;
                    if (kLinked) {   // the next block starts from this table: no ip-2 fill after a match
                        // ending past mflimit (lz4.c:1142-1146)
                        const bool endm = Mm && base + eL >= mfe;
                        restore(endm && eL - 2 < LZH_WAVE ? I & ~(1ull << (eL - 2)) : I);
                    }
                } else {
                    // table: the last inserted lane of each slot, or the slot's old value
                    const bool inI = lane_on(I);
                    if (LZH_LZ4_RESTORE2 && !losers) {
                        // (no two lanes share a slot: every claim stands, a lane not inserted puts its old value back)
                        if (valid && !inI) T.put(h, old);
                    } else if (vmask == ~0ull) {
                        // every lane stores its slot's final value (all lanes of a slot agree):
                        // the slot's last inserted lane, else its old value
                        const uint64_t gi = grp & I;
                        T.put(h, gi ? (uint32_t)(base + 63 - __builtin_clzll(gi)) : old);
                    } else if (!losers) {
                        if (valid && !inI) T.put(h, old);
                    } else {
                        const uint64_t gi = grp & I;
                        const bool wr = valid && (gi == 0 || (inI && (gi & ~((2ull << lane) - 1ull)) == 0));
                        if (wr) T.put(h, inI ? (uint32_t)p : old);
                    }
                    wave_lds_fence();
                }
                // the loop state, after the parse's last batch too (the parse then reads only anchor, whose
                // update is the same): one path into the back edge for the state, no copies merging an
                // unchanged branch
                const int swc = !Mm && hi0 == qlim - base;             // 64 probes done: stride batches
                if (Mm) {
                    const int ip = base + eL;
                    anchor = ip;
                    so = ip;
                    if (eL < LZH_WAVE) {                               // searched to the batch end
                        q = base + LZH_WAVE;
                        qlim = ip + dlim;
                        pins = -1;
                    } else {                                           // re-test in a later batch
                        q = ip;
                        qlim = ip + dlim;
                        pins = eL - 2 >= LZH_WAVE ? ip - 2 : -1;
                    }
                } else {
                    q = base + hi0 + 1;
                    pins = -1;
                }
                if (swc) {
                    if (LZH_LZ4_SWP) {
                        runb = 2;   // (the switch itself at the next batch's head: off the run batches' back edge)
                    } else {
                        runb = 0;
                        s = so + 1;
                        k0 = LZH_WAVE;
                        retest = 0;
                    }
                } else {
                    base = pins >= 0 ? pins : q;
                }
                __builtin_amdgcn_s_setprio(0);
                LZ_CLK(8);                                             // table restore
                continue;
            }

            // ================= stride batch: first sequence only
            // (the run path's deferred record fields are consumed by now: fresh values here too, so the batch loop's
            // back edge needs no VGPR copies to merge the run and stride paths' values)
            if (LZH_LZ4_PRFRESH) { pr_e = 0; pr_cn = 0; pr_be = 0; pr_ce = 0; }
            uint64_t hits = ballot(ok);
            const uint64_t tmask = ballot(!valid);
            const int fi = ffs64(tmask);
            int fh = ffs64(hits);
            bool found = hits != 0;
            int L = found ? fh : fi - 1;
            uint64_t upto = L < 0 ? 0ull : (L >= 63 ? ~0ull : ((2ull << L) - 1ull));
            if (!(losers & upto)) {
                if (valid && lane > L && back == (uint32_t)p) T.put(h, old);
            } else {
                // lanes up to L sharing a slot: each sees the previous lane of its slot
                LZ_STAT(1, 1);
                if (valid) T.put(h, old);
                wave_lds_fence();
                uint64_t grp;
                int prev;
                slot_groups(h, valid, losers, grp, prev, lane);
                const uint32_t ppos = lane_gather((uint32_t)p, prev < 0 ? lane : prev);
                if (prev >= 0) cand = ppos;
                W.load(in, cand, valid);
                wait_vm();
                R.ready = R.fill;
                ok = eval_lane(ps, W, valid, bkr, len);
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
            wave_lds_fence();
            // (uniform: a phi of `found` the compiler takes as divergent turns the whole batch loop's
            // state into VGPR copies read back by readfirstlane at every iteration)
            found = unii(found) != 0; fh = unii(fh);
            if (!found) {
                if (tmask) go = 0;                                 // ran past mflimit
                else if (retest) { retest = 0; k0 = LZH_WAVE - 1; }
                else k0 += LZH_WAVE;
            } else {
                LZ_STAT(3, 1);
                const int P = rdlanei(p, fh);
                const int M = rdlanei((int)cand, fh);
                int cnt;
                int bk = finish_match<kStats>(in, P, M, kRec ? 0 : rdlanei(bkr, fh), rdlanei(len, fh), anchor, mlimit,
                                              cnt, lane, ctr);
                if (kRec) bk = 0;   // (catch-up in the emission kernel)
                {
                    const int lit = P - bk - anchor, mlx = bk + cnt;
                    rc_anc = (uint32_t)anchor;
                    rc_p = (uint32_t)P;
                    rc_lit = kRec ? (uint32_t)P : (uint32_t)lit;   // kRec: the match start P
                    rc_off = (uint32_t)(P - M);
                    rc_mlx = (uint32_t)mlx;
                    rc_st = 0;
                    rc_m = 1;
                    rc_tot = 3 + lit + ext_len_bytes(lit) + ext_len_bytes(mlx);
                }
                const int ip = P + kMinMatch + cnt;
                anchor = ip;
                if (ip >= mfe) {
                    go = 0;
                } else if (acc == 1 || kFast) {                        // back to run batches
                    runb = 1;
                    pins = ip - 2;
                    base = ip - 2;
                    q = ip;
                    so = ip;
                    qlim = ip + dlim;
                } else {   // fill table at ip-2 (lz4.c:1146), then re-test ip as lane 0
                    uint32_t w, bb = 0;
                    if (R.has(ip - 6, ip + 8)) { w = R.u32(ip - 2); if (!kSmall) bb = R.byte(ip + 2); }
                    else { const uint64_t v = in.w40(ip - 2); w = (uint32_t)v; bb = (uint32_t)(v >> 32); }
                    const uint32_t hm2 = hash_of<kSmall>(w, bb);
                    if (lane == 0) T.put(hm2, (uint32_t)(ip - 2));
                    wave_lds_fence();
                    retest = 1;
                    s = ip + 1;
                    k0 = 0;
                }
            }
        }
    }
    wait_vm();
    R.ready = R.fill;
    wave_lds_fence();
    if (!aborted) {
        RUN_RECORDS();
        RECS_OUT();
    }
    if (kRec) {
        if (lane == 0) { rec_hdr[0] = (uint32_t)nrec; rec_hdr[1] = (uint32_t)anchor; }
    } else {
        const int run = b0 + n - anchor;
        if (kLinked && !aborted && op + run + 1 + (run + 240) / 255 > lk->cap) {   // last literals (lz4.c:1207-1216)
            lk->abort = -2;
            aborted = true;
        }
        if (kLinked && aborted) {   // the block is stored raw: nothing to emit
            if (lane == 0 && out_size) *out_size = (uint32_t)n;
        } else {
            if (op - O.flushed >= 4 * LZH_WAVE) O.flush(out, ((op + O.sh) & ~3) - O.sh, lane);
            op = emit_seq(in, R, out, O, op, anchor, run, false, 0, 0, lane);
            O.flush(out, op, lane);
            if (lane == 0 && out_size) *out_size = (uint32_t)op;
        }
    }
    if (kStats && lane == 0) {
        for (int i = 0; i < kCtr; i++) atomicAdd(&stats[i], (unsigned long long)ctr[i]);
        for (int i = 0; i < kClk; i++) atomicAdd(&stats[13 + i], (unsigned long long)clk[i]);
    }
}

}  // namespace lz4v3

extern "C" __global__ void __launch_bounds__(64)
lzh_lz4_compress_v2_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size, int acc,
                           uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t chunk0,
                           unsigned long long* stats) {
    // table 16 KiB | input ring 1 KiB | output ring 512 B  (17.5 KiB: 9 waves per CU)
    __shared__ __attribute__((aligned(16))) uint32_t lds[4096 + lz4v3::kRing / 4 + lz4v3::kOut / 4];
    const uint64_t chunk = (uint64_t)blockIdx.x + chunk0;
    const uint64_t off = chunk * chunk_size;
    if (off >= n_total && !(n_total == 0 && chunk == 0)) return;
    const int n = (int)min(chunk_size, n_total - off);
    const uint64_t readable = min<uint64_t>(in_readable - off, (uint64_t)n + 64);
    Bytes rin, rout;
    rin.init(in + off, readable);
    rout.init(stage + chunk * stride, stride);
    LDSA uint32_t* tab = (LDSA uint32_t*)lds;
    LDSA uint32_t* ring = tab + 4096;
    LDSA uint8_t* outb = (LDSA uint8_t*)(ring + lz4v3::kRing / 4);
    const rsrc_t nr = make_rsrc(nullptr, 0);
    if (n < 65547) {
        if (acc > 1) lz4v3::compress_chunk<true, false, false, true>(rin, n, rout, acc, tab, ring, outb, csizes + chunk, stats, nr, nullptr);
        else lz4v3::compress_chunk<true, false>(rin, n, rout, acc, tab, ring, outb, csizes + chunk, stats, nr, nullptr);
    } else {
        if (acc > 1) lz4v3::compress_chunk<false, false, false, true>(rin, n, rout, acc, tab, ring, outb, csizes + chunk, stats, nr, nullptr);
        else lz4v3::compress_chunk<false, false>(rin, n, rout, acc, tab, ring, outb, csizes + chunk, stats, nr, nullptr);
    }
}

// debug twin of the parse kernel with event counters and phase clocks (tools/lz4_stats.py)
extern "C" __global__ void __launch_bounds__(64)
lzh_lz4_compress_stats_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size, int acc,
                              uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t chunk0,
                              unsigned long long* stats) {
    // (the parse kernel's path: records dropped by a zero-size descriptor, header into LDS scratch)
    __shared__ __attribute__((aligned(16))) uint32_t lds[4096 + lz4v3::kRing / 4 + 8];
    __shared__ uint32_t hdr[2];
    const uint64_t chunk = (uint64_t)blockIdx.x + chunk0;
    const uint64_t off = chunk * chunk_size;
    if (off >= n_total && !(n_total == 0 && chunk == 0)) return;
    const int n = (int)min(chunk_size, n_total - off);
    const uint64_t readable = min<uint64_t>(in_readable - off, (uint64_t)n + 64);
    Bytes rin, rout;
    rin.init(in + off, readable);
    rout.init(stage + chunk * stride, stride);
    LDSA uint32_t* tab = (LDSA uint32_t*)lds;
    LDSA uint32_t* ring = tab + 4096;
    const rsrc_t nr = make_rsrc(nullptr, 0);
    if (n < 65547) {
        if (acc > 1) lz4v3::compress_chunk<true, true, true, true, false, LZH_LZ4_RW>(rin, n, rout, acc, tab, ring, nullptr, nullptr, stats, nr, hdr);
        else lz4v3::compress_chunk<true, true, true, false, false, LZH_LZ4_RW>(rin, n, rout, acc, tab, ring, nullptr, nullptr, stats, nr, hdr);
    } else {
        if (acc > 1) lz4v3::compress_chunk<false, true, true, true, false, LZH_LZ4_RW>(rin, n, rout, acc, tab, ring, nullptr, nullptr, stats, nr, hdr);
        else lz4v3::compress_chunk<false, true, true, false, false, LZH_LZ4_RW>(rin, n, rout, acc, tab, ring, nullptr, nullptr, stats, nr, hdr);
    }
}

// ======================================================================= parse + emit split
// The parse kernel (one wave per chunk, the compress_chunk loop above with kRec) leaves every
// sequence as an 8-byte record; lzh_lz4_emit_kernel, which needs no hash table and runs at high
// occupancy, lays the LZ4 block out (lz4.c:1022-1135 sequence format, :1204-1231 last literals):
// for 64 records at a time a wave computes input anchors and output offsets by prefix sums,
// every lane writes its sequence's bytes into an LDS ring, and the ring leaves for the staging
// slot as aligned dwords.  Chunks up to 16 MiB (24-bit literal / match-length fields).

extern "C" __global__ void __launch_bounds__(64)
lzh_lz4_parse_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size, int acc,
                     uint8_t* recs, uint64_t rec_stride, uint32_t* rec_hdr, uint64_t frame_size, uint32_t bpf) {
    // table only (the P sides from a register window, compress_chunk's kRW)
    // (LZH_LZ4_PADLDS: extra bytes of LDS per wave -- an occupancy experiment, 0 in builds)
    __shared__ __attribute__((aligned(16))) uint32_t lds[4096 + (LZH_LZ4_RW ? 0 : lz4v3::kRing / 4 + 8) + LZH_LZ4_PADLDS / 4];
    const uint64_t chunk = blockIdx.x;
    uint64_t off;
    int n;
    if (!block_span(chunk, n_total, chunk_size, frame_size, bpf, off, n)) return;
    const uint64_t readable = min<uint64_t>(in_readable - off, (uint64_t)n + 64);
    Bytes rin, rout;
    rin.init(in + off, readable);
    rout.init(nullptr, 0);
    LDSA uint32_t* tab = (LDSA uint32_t*)lds;
    LDSA uint32_t* ring = tab + 4096;
    const rsrc_t rr = make_rsrc(recs + chunk * rec_stride, (uint32_t)rec_stride);
    uint32_t* hdr = rec_hdr + 2 * chunk;
    if (n < 65547) {
        if (acc > 1) lz4v3::compress_chunk<true, false, true, true, false, LZH_LZ4_RW>(rin, n, rout, acc, tab, ring, nullptr, nullptr, nullptr, rr, hdr);
        else lz4v3::compress_chunk<true, false, true, false, false, LZH_LZ4_RW>(rin, n, rout, acc, tab, ring, nullptr, nullptr, nullptr, rr, hdr);
    } else {
        if (acc > 1) lz4v3::compress_chunk<false, false, true, true, false, LZH_LZ4_RW>(rin, n, rout, acc, tab, ring, nullptr, nullptr, nullptr, rr, hdr);
        else lz4v3::compress_chunk<false, false, true, false, false, LZH_LZ4_RW>(rin, n, rout, acc, tab, ring, nullptr, nullptr, nullptr, rr, hdr);
    }
}

namespace lz4e {

constexpr int kRingB = 2048;            // LDS output ring (bytes)
constexpr int kSpan = 2048;             // LDS copy of a record group's input span (bytes)
// (4 KiB of LDS per wave: the emission kernel runs at the full 8 waves per SIMD)
// longest literal run the lane-parallel group layout takes (<= 269: one literal-length byte)
#ifndef LZH_LZ4E_LITMAX
#define LZH_LZ4E_LITMAX 255   // (64 -> 255: emit 1.28 -> 1.21 ms per GiB of text, profiles/r03_c/ab.txt)
#endif

__device__ __forceinline__ int wave_max(int v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
    return v;
}

__device__ __forceinline__ int ext_len(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

// bytes [p-4, p) as a dword, byte p-1 the most significant; bytes before 0 read as 0
__device__ __forceinline__ uint32_t u32_before(const Bytes& in, int p) {
    if (p >= 4) return in.w32(p - 4);
    return p <= 0 ? 0u : in.w32(0) << (8 * (4 - p));
}
__device__ __forceinline__ int wave_excl_scan(int x, int lane, int& total) {
    int incl = lz4v3::wave_incl_scan(x);
    total = __builtin_amdgcn_readlane(incl, 63);
    return incl - x;
}

struct OutR {
    LDSA uint8_t* b;
    rsrc_t o;          // staging slot (256-aligned)
    int flushed;       // bytes [0, flushed) are in global memory
    __device__ __forceinline__ void put(int pos, uint32_t v) const { ((volatile LDSA uint8_t*)b)[pos & (kRingB - 1)] = (uint8_t)v; }
    // global <- complete dwords of [flushed, upto) (all of it when fin: the partial last dword too)
    __device__ __forceinline__ void flush(int upto, bool fin, int lane) {
        wave_lds_fence();
        const int d0 = flushed >> 2, d1 = fin ? (upto + 3) >> 2 : upto >> 2;
        for (int d = d0 + lane; d < d1; d += 64)
            st_b32(o, 4 * d, ((volatile LDSA uint32_t*)b)[d & (kRingB / 4 - 1)]);
        flushed = 4 * d1;
        if (flushed > upto) flushed = upto & ~3;   // (the partial dword is rewritten by the next flush)
        wave_lds_fence();
    }
};

// One group of 64 records: its header (sequences before catch-up; the literals of a record run from
// the previous record's match end, lane-1 by a wave shift, the previous group's end for lane 0).
// Its loads -- the dwords under the catch-up words before the match and its candidate, and the
// group's input span [ia, ia + Lt) -- go into the caller's registers, issued a group ahead of use,
// unconditionally (out-of-range buffer reads return 0): a load under a branch merges with the old
// register value, and that copy would wait for the load.
constexpr int kSpanW = kSpan / 256;     // span dwords per lane
struct Grp {
    int Pm = 0, mlx = 0, o = 0, anc = 0, lit = 0, ia = 0, Lt = 0, X0 = 0, nd = 0;
    bool v = false, span = false;
    __device__ __forceinline__ void head(uint32_t w0, uint32_t w1, int ia_, int g, int nrec, const Bytes& in, int lane) {
        v = g + lane < nrec;
        Pm = (int)(w0 & 0xFFFFFFu);
        mlx = (int)((w0 >> 24) | ((w1 & 0xFFFFu) << 8));
        o = (int)(w1 >> 16);
        const int end = Pm + 4 + mlx;
        ia = ia_;
        anc = __builtin_amdgcn_update_dpp(ia_, end, 0x138, 0xf, 0xf, false);   // wave_shr:1
        lit = Pm - anc;
        const int nv = max(min(64, nrec - g), 1);
        Lt = __builtin_amdgcn_readlane(end, nv - 1) - ia_;
        span = Lt + 8 <= kSpan;
        X0 = (ia_ + in.sh) & ~3;
        nd = (ia_ + in.sh + Lt - X0 + 3) >> 2;
    }
    // raw dwords: c[0..1] under bytes [Pm-4, Pm), c[2..3] under [M-4, M) (M = Pm - o), span words
    __device__ __forceinline__ void issue(const Bytes& in, int lane, uint32_t* c, uint32_t* sp) const {
        // (words nobody needs re-read the group's first span dword: no extra memory traffic)
        const int a0 = X0 + 4 * lane;
        const bool cu = v && min(lit, Pm - o) > 0;
        const int xp = cu ? (max(Pm - 4, 0) + in.sh) & ~3 : a0, xm = cu ? (max(Pm - o - 4, 0) + in.sh) & ~3 : a0;
        c[0] = ld_b32(in.r, xp); c[1] = ld_b32(in.r, xp + 4);
        c[2] = ld_b32(in.r, xm); c[3] = ld_b32(in.r, xm + 4);
#pragma unroll
        for (int k = 0; k < kSpanW; k++) sp[k] = ld_b32(in.r, span && 64 * k < nd ? a0 + 256 * k : a0);
    }
    // the dword of bytes [p-4, p), byte p-1 most significant, bytes before 0 as 0 (u32_before)
    __device__ __forceinline__ static uint32_t before(uint32_t lo, uint32_t hi, int p, int sh) {
        const uint32_t w = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)(max(p - 4, 0) + sh) & 3u);
        return p >= 4 ? w : (p <= 0 ? 0u : w << (8 * (4 - p)));
    }
};

// bytes of one sequence (or the last literals: ml < 0) written by the whole wave through the ring
__device__ void put_seq_wave(OutR& R, const Bytes& in, int op, int anchor, int lit, int off, int mlx, int lane) {
    const bool hm = mlx >= 0;
    const int lx = ext_len(lit), mx = hm ? ext_len(mlx) : 0;
    const uint32_t token = ((uint32_t)min(lit, 15) << 4) | (hm ? (uint32_t)min(mlx, 15) : 0u);
    int pos = op;
    if (lane == 0) R.put(pos, token);
    pos++;
    for (int b = 0; b < lx; b += 64) {
        if (pos + b - R.flushed >= kRingB - 128) R.flush(pos + b, false, lane);
        if (b + lane < lx) R.put(pos + b + lane, b + lane == lx - 1 ? (uint32_t)(lit - 15) % 255u : 255u);
    }
    pos += lx;
    if (lit >= 256) {   // long literal run (incompressible data, last literals): straight to HBM
        bulk_literals<kRingB>(R, in, anchor, pos, lit, lane);
    } else {
        for (int b = 0; b < lit; b += 64) {
            if (pos + b - R.flushed >= kRingB - 128) R.flush(pos + b, false, lane);
            if (b + lane < lit) R.put(pos + b + lane, in.b(anchor + b + lane));
        }
    }
    pos += lit;
    if (hm) {
        if (pos - R.flushed >= kRingB - 128) R.flush(pos, false, lane);
        if (lane < 2) R.put(pos + lane, lane ? ((uint32_t)off >> 8) : ((uint32_t)off & 0xffu));
        pos += 2;
        for (int b = 0; b < mx; b += 64) {
            if (pos + b - R.flushed >= kRingB - 128) R.flush(pos + b, false, lane);
            if (b + lane < mx) R.put(pos + b + lane, b + lane == mx - 1 ? (uint32_t)(mlx - 15) % 255u : 255u);
        }
    }
}

}  // namespace lz4e

// (8 waves per SIMD: the group pipeline's registers fit 64 VGPRs without spills; left to itself the
// compiler takes 66 and 7 waves)
#ifndef LZH_EMIT_WAVES
#define LZH_EMIT_WAVES 8
#endif
extern "C" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LZH_EMIT_WAVES, 8)))
lzh_lz4_emit_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                    const uint8_t* recs, uint64_t rec_stride, const uint32_t* rec_hdr, uint8_t* stage, uint64_t stride,
                    uint32_t* csizes, uint64_t frame_size, uint32_t bpf) {
    __shared__ __attribute__((aligned(16))) uint8_t ring[lz4e::kRingB];
    __shared__ __attribute__((aligned(16))) uint32_t ibuf[lz4e::kSpan / 4 + 4];   // input span of a group
    const int lane = threadIdx.x;
    const uint64_t chunk = blockIdx.x;
    uint64_t off;
    int n;
    if (!block_span(chunk, n_total, chunk_size, frame_size, bpf, off, n)) return;
    Bytes in_b;
    in_b.init(in + off, min<uint64_t>(in_readable - off, (uint64_t)n + 64));
    const rsrc_t rr = make_rsrc(recs + chunk * rec_stride, (uint32_t)rec_stride);
    const int nrec = (int)uni(rec_hdr[2 * chunk]);
    lz4e::OutR R{(LDSA uint8_t*)ring, make_rsrc(stage + chunk * stride, (uint32_t)stride), 0};
    // Software pipeline over groups of 64 records: while group g is laid out, the loads of group g+1
    // (its input span and catch-up words) and the records of group g+2 are in flight, so a group's one
    // memory wait comes a whole group after its loads were issued.
    int op = 0, ia_end = 0;
    lz4e::Grp GA, GB;                           // headers of groups g and g+1 (alternating roles)
    uint32_t sp[lz4e::kSpanW], cw[4];           // group g's span and catch-up dwords (in flight)
    // records of group g+1 (in flight), per lane; past nrec the offsets are out of range (0)
    uint32_t nw0 = ld_b32(rr, 8 * (64 + lane)), nw1 = ld_b32(rr, 8 * (64 + lane) + 4);
    {
        const uint32_t w0 = ld_b32(rr, 8 * lane), w1 = ld_b32(rr, 8 * lane + 4);
        GA.head(w0, w1, 0, 0, nrec, in_b, lane);
        GA.issue(in_b, lane, cw, sp);
    }
    auto step = [&](lz4e::Grp& G, lz4e::Grp& Gn, int g) {
        // group g's input span into LDS (literal bytes are read from it), its catch-up words
        if (G.span) {
#pragma unroll
            for (int k = 0; k < lz4e::kSpanW; k++)
                if (64 * k < G.nd && lane + 64 * k < G.nd) ibuf[lane + 64 * k] = sp[k];
            wave_lds_fence();
        }
        const uint32_t xp = lz4e::Grp::before(cw[0], cw[1], G.Pm, in_b.sh);
        const uint32_t xm = lz4e::Grp::before(cw[2], cw[3], G.Pm - G.o, in_b.sh);
        // group g+1: header from its records; its loads and the records of group g+2 go out now
        {
            const uint32_t w0 = nw0, w1 = nw1;
            nw0 = ld_b32(rr, 8 * (g + 128 + lane));
            nw1 = ld_b32(rr, 8 * (g + 128 + lane) + 4);
            Gn.head(w0, w1, G.ia + G.Lt, g + 64, nrec, in_b, lane);
            Gn.issue(in_b, lane, cw, sp);
        }
        const bool v = G.v;
        int lit = G.lit, mlx = G.mlx;
        const int Pm = G.Pm, o = G.o, anc = G.anc, ia = G.ia, Lt = G.Lt;
        const bool span = G.span;
        const int X0 = G.X0;
        int T;
        const int M = Pm - o;
        const int maxb = min(lit, M);
        if (v && maxb > 0) {   // catch-up (lz4.c:1017-1020): extend the match backwards while ip > anchor, match > start
            const uint32_t x = xp ^ xm;
            int bk = x ? (int)((uint32_t)__builtin_clz(x) >> 3) : 4;
            bk = min(bk, maxb);
            if (bk == 4) {                                   // (rare) past the first 4 bytes
                while (bk < maxb && in_b.b(Pm - 1 - bk) == in_b.b(M - 1 - bk)) bk++;
            }
            lit -= bk;
            mlx += bk;
        }
        const int S = v ? 3 + lit + lz4e::ext_len(lit) + lz4e::ext_len(mlx) : 0;
        const int pos = op + lz4e::wave_excl_scan(S, lane, T);
        const int litv = v ? lit : 0;
        const int litmax = (int)uni((uint32_t)lz4e::wave_max(litv));
        if (T <= lz4e::kRingB / 2 && litmax <= LZH_LZ4E_LITMAX && span) {
            const LDSA uint8_t* ib = (const LDSA uint8_t*)ibuf;
            const int ioff = ia + in_b.sh - X0 - ia;   // input position p lives at ib[p + ioff]
            // every lane writes its own sequence (lz4.c:1022-1135): token, one literal-length byte
            // when lit >= 15 (lit <= LZH_LZ4E_LITMAX <= 269 here), the literals (a lane-parallel copy as long as the
            // group's longest run), offset, match-length bytes
            if (op + T - R.flushed > lz4e::kRingB - 8) R.flush(op, false, lane);
            const int lx = lz4e::ext_len(lit), mx = lz4e::ext_len(mlx);
            const uint32_t token = ((uint32_t)min(lit, 15) << 4) | (uint32_t)min(mlx, 15);
            const int lp = pos + 1 + lx;
            if (v) {
                R.put(pos, token);
                if (lx) R.put(pos + 1, (uint32_t)(lit - 15));
            }
            for (int t = 0; t < litmax; t++)
                if (t < litv) R.put(lp + t, ib[anc + t + ioff]);
            const int mp = lp + lit;
            if (v) {
                R.put(mp, (uint32_t)o & 0xffu);
                R.put(mp + 1, (uint32_t)o >> 8);
            }
            for (int t = 0; ballot(v && t < mx); t++)
                if (v && t < mx) R.put(mp + 2 + t, t == mx - 1 ? (uint32_t)(mlx - 15) % 255u : 255u);
            op += T;
            if (op - R.flushed >= lz4e::kRingB / 2) R.flush(op, false, lane);
            wave_lds_fence();
        } else {
            for (int k = 0; k < 64 && g + k < nrec; k++) {
                const int kl = rdlanei(lit, k), km = rdlanei(mlx, k), ko = rdlanei(o, k), ka = rdlanei(anc, k);
                if (op + 256 - R.flushed > lz4e::kRingB) R.flush(op, false, lane);
                lz4e::put_seq_wave(R, in_b, op, ka, kl, ko, km, lane);
                op += 3 + kl + lz4e::ext_len(kl) + lz4e::ext_len(km);
            }
        }
        ia_end = ia + Lt;
    };
    for (int g = 0; g < nrec; g += 128) {
        step(GA, GB, g);
        if (g + 64 < nrec) step(GB, GA, g + 64);
    }
    const int ia = ia_end;
    // last literals (lz4.c:1204-1231): everything after the last match, the whole chunk if none
    const int last = n - ia;
    if (op + 256 - R.flushed > lz4e::kRingB) R.flush(op, false, lane);
    lz4e::put_seq_wave(R, in_b, op, ia, last, 0, -1, lane);
    op += 1 + last + lz4e::ext_len(last);
    R.flush(op, true, lane);
    if (lane == 0) csizes[chunk] = (uint32_t)op;
}

#ifndef LZH_NO_LINKED_KERNEL
// LZ4 frames with linked blocks (LZ4F_blockLinked, the LZ4F default; lz4frame.c:651-655, :777-782):
// one wave per frame walks its blocks in order with one byU32 table, as LZ4_compress_fast_continue
// does over a stable source (lz4.c:1565-1628, prefix mode).  Each block is compressed with the
// limitedOutput budget size - 1 (LZ4F_makeBlock, lz4frame.c:740-763); a block that does not fit is
// stored raw (bcs = its size) and its table is rebuilt as the reference leaves it at the failing
// check: the table is saved to `snap` (16 KiB per frame) before every block and a failed block is
// replayed from it up to the failing probe.  A frame of one block is independent (lz4frame.c:394-395)
// and goes through the chunk codec.  Block i of frame f: staging slot f * bpf + b, size bcs[i].
template <bool kFast>
__device__ void lz4f_linked_frame(const Bytes& rin, uint64_t s, uint64_t bs, uint32_t bpf, uint64_t f, int acc,
                                  uint8_t* stage, uint64_t stride, uint32_t* bcs, uint32_t* snap, LDSA uint32_t* tab,
                                  LDSA uint32_t* ring, LDSA uint8_t* outb) {
    const int lane = threadIdx.x;
    const rsrc_t nr = make_rsrc(nullptr, 0);
    const uint32_t nb = (uint32_t)((s + bs - 1) / bs);
    const rsrc_t sn = make_rsrc(snap + f * 4096, 16384);
    for (uint32_t b = 0; b < nb; b++) {
        const int b0 = (int)(b * bs), bn = (int)min<uint64_t>(bs, s - b * bs);
        const uint64_t i = f * bpf + b;
        if (b > 0) {   // the table before this block (a failed block replays from it)
            wave_lds_fence();
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const int d = 4 * (k * LZH_WAVE + lane);
                const u32x4 v = {tab[d], tab[d + 1], tab[d + 2], tab[d + 3]};
                __builtin_amdgcn_raw_buffer_store_b128(v, sn, 4 * d, 0, 0);
            }
        }
        Bytes rout;
        rout.init(stage + i * stride, stride);
        lz4v3::LinkCtl L{b0, bn - 1, -1, b > 0, -1};
        lz4v3::compress_chunk<false, false, false, kFast, true>(rin, bn, rout, acc, tab, ring, outb, bcs + i,
                                                                        nullptr, nr, nullptr, &L);
        if (L.abort >= 0) {   // replay up to the failing probe: the table the next block starts from
            if (b > 0) {
                wait_vm();
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const int d = 4 * (k * LZH_WAVE + lane);
                    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(sn, 4 * d, 0, 0);
                    tab[d] = v[0]; tab[d + 1] = v[1]; tab[d + 2] = v[2]; tab[d + 3] = v[3];
                }
                wave_lds_fence();
            }
            Bytes nul;
            nul.r = nr;
            nul.sh = 0;
            lz4v3::LinkCtl Rp{b0, 0x7fffffff, L.abort, b > 0, -1};
            lz4v3::compress_chunk<false, false, false, kFast, true>(rin, bn, nul, acc, tab, ring, outb, nullptr,
                                                                            nullptr, nr, nullptr, &Rp);
        }
        wave_lds_fence();
    }
}

extern "C" __global__ void __launch_bounds__(64)
lzh_lz4f_linked_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t fs, uint64_t bs, uint32_t bpf,
                       int acc, uint8_t* stage, uint64_t stride, uint32_t* bcs, uint32_t* snap) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4096 + lz4v3::kRing / 4 + lz4v3::kOut / 4];
    const uint64_t f = blockIdx.x;
    const uint64_t foff = f * fs;
    if (foff >= n_total) return;
    const uint64_t s = min(fs, n_total - foff);
    Bytes rin;
    rin.init(in + foff, min<uint64_t>(in_readable - foff, s + 64));
    LDSA uint32_t* tab = (LDSA uint32_t*)lds;
    LDSA uint32_t* ring = tab + 4096;
    LDSA uint8_t* outb = (LDSA uint8_t*)(ring + lz4v3::kRing / 4);
    if (s <= bs) {   // one block: independent (the chunk codec with its own table type)
        const rsrc_t nr = make_rsrc(nullptr, 0);
        Bytes rout;
        rout.init(stage + f * bpf * stride, stride);
        uint32_t* cs = bcs + f * bpf;
        const int n = (int)s;
        if (n < 65547) {
            if (acc > 1) lz4v3::compress_chunk<true, false, false, true>(rin, n, rout, acc, tab, ring, outb, cs, nullptr, nr, nullptr);
            else lz4v3::compress_chunk<true, false>(rin, n, rout, acc, tab, ring, outb, cs, nullptr, nr, nullptr);
        } else {
            if (acc > 1) lz4v3::compress_chunk<false, false, false, true>(rin, n, rout, acc, tab, ring, outb, cs, nullptr, nr, nullptr);
            else lz4v3::compress_chunk<false, false>(rin, n, rout, acc, tab, ring, outb, cs, nullptr, nr, nullptr);
        }
        return;
    }
    if (acc > 1) lz4f_linked_frame<true>(rin, s, bs, bpf, f, acc, stage, stride, bcs, snap, tab, ring, outb);
    else lz4f_linked_frame<false>(rin, s, bs, bpf, f, acc, stage, stride, bcs, snap, tab, ring, outb);
}

#endif
#include "launch.h"
size_t lzh_lz4_rec_stride(uint64_t chunk_size) { return ((chunk_size / 4 + 4) * 8 + 255) / 256 * 256; }

hipError_t lzh_launch_lz4_compress_v2(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                      int acc, uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks,
                                      hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(lzh_lz4_compress_v2_kernel, dim3(nchunks), dim3(64), 0, s, in, n_total, in_readable,
                       chunk_size, acc, stage, stride, csizes, 0u, (unsigned long long*)nullptr);
    return hipGetLastError();
}

// parse kernel + emit kernel (records in `recs`: nchunks x rec_stride bytes, then 8 bytes per chunk);
// stage_mask bit 0 = parse, bit 1 = emit (profiling runs one of them)
hipError_t lzh_launch_lz4_split(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size, int acc,
                                uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks, uint8_t* recs,
                                int stage_mask, hipStream_t s, uint64_t frame_size, uint32_t bpf) {
    if (nchunks == 0) return hipSuccess;
    if (bpf <= 1) { bpf = 1; frame_size = chunk_size; }
    const uint64_t rs = lzh_lz4_rec_stride(chunk_size);
    uint32_t* hdr = (uint32_t*)(recs + rs * nchunks);
    if (stage_mask & 1)
        hipLaunchKernelGGL(lzh_lz4_parse_kernel, dim3(nchunks), dim3(64), 0, s, in, n_total, in_readable, chunk_size,
                           acc, recs, rs, hdr, frame_size, bpf);
    if (stage_mask & 2)
        hipLaunchKernelGGL(lzh_lz4_emit_kernel, dim3(nchunks), dim3(64), 0, s, in, n_total, in_readable, chunk_size,
                           (const uint8_t*)recs, rs, (const uint32_t*)hdr, stage, stride, csizes, frame_size, bpf);
    return hipGetLastError();
}

hipError_t lzh_launch_lz4f_linked(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t fs, uint64_t bs,
                                  uint32_t bpf, int acc, uint8_t* stage, uint64_t stride, uint32_t* bcs, uint32_t* snap,
                                  uint32_t nframes, hipStream_t s) {
    if (nframes == 0) return hipSuccess;
#ifdef LZH_NO_LINKED_KERNEL
    return hipErrorNotSupported;
#else
    hipLaunchKernelGGL(lzh_lz4f_linked_kernel, dim3(nframes), dim3(64), 0, s, in, n_total, in_readable, fs, bs, bpf, acc,
                       stage, stride, bcs, snap);
    return hipGetLastError();
#endif
}

// debug: run the v2 kernel with event counters (16 x u64 device buffer)
extern "C" int lzh_debug_lz4_stats(const void* d_in, uint64_t n, uint64_t in_readable, uint64_t chunk_size, int acc,
                                   void* d_stage, uint32_t* d_csizes, unsigned long long* d_stats, void* stream) {
    const uint64_t k = (n + chunk_size - 1) / chunk_size;
    const uint64_t stride = ((chunk_size + chunk_size / 255 + 16 + 16) + 255) / 256 * 256;
    hipLaunchKernelGGL(lzh_lz4_compress_stats_kernel, dim3((unsigned)k), dim3(64), 0, (hipStream_t)stream,
                       (const uint8_t*)d_in, n, in_readable, chunk_size, acc, (uint8_t*)d_stage, stride, d_csizes, 0u,
                       d_stats);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}
