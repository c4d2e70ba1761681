// lzbench_amd/csrc/zstdc_hip.hip -- zstd 1.5.2 frame compression for gfx950 (the hip_zstd row),
// bit-exact with the reference build for the fast-strategy levels lzbench's zstd rows use
// (zstd -1 / -2 where fast, zstd_fast -1..-5; reference _lzbench/compressors.cpp:1745-1770:
// ZSTD_getParams(level, part, 0) + contentSizeFlag + ZSTD_compress_advanced).
//
// One frame per chunk.  A frame is processed block by block (blocks of min(128 KiB, 2^windowLog),
// zstd_compress.c:3932-4009), each block by two kernels:
//
//   lzh_zstd_match_kernel    one wave per frame: the fast match finder of zstd_fast.c:92-315 on
//                            the block, hash table in LDS (or in the frame's scratch when it does
//                            not fit), sequences + literals to the frame's scratch.
//   lzh_zstd_entropy_kernel  one wave per frame: literals (Huffman, zstd_compress_literals.c /
//                            huf_compress.c), sequences (FSE, zstd_compress_sequences.c), the
//                            raw / RLE / compressed block decision (zstd_compress.c:3762-3824),
//                            frame header; appends the block to the frame's staging slot.
//
// The split per block is what the format needs: a block emitted raw or RLE does not confirm its
// repcodes (zstd_compress.c:3813), so block k+1's parse starts from repcodes only the entropy
// stage of block k knows.  Single-block frames (-b64, -b128) take one launch of each kernel.
//
// Match finder on a 64-lane wave.  From a search start the reference probes positions in pairs
// (A, A+1), the pair start advancing by a step that grows every 128 bytes, and checks the
// repcode at A+D before the pair's own hash matches; each probed position reads its hash slot
// and then overwrites it.  A batch evaluates 32 pairs at once (lane 2j: A_j, lane 2j+1: A_j+1):
// every lane reads its slot, claims it, reads the claim back -- lanes sharing a slot are grouped
// by the claim winner -- and takes as candidate the closest earlier lane of its group (that lane
// was probed before it) or the slot's old value.  The first event in probe order (repcode of
// pair j, hit at A_j, hit at A_j+1) ends the batch; slots are then rewritten to the value the
// sequential order leaves: the last probed member of each group, or the old value.
#include "common.h"

namespace zc {

// ------------------------------------------------------------------ parameters (host + device)
struct ZParams {
    int ok;
    uint32_t wlog, hlog, mls, tlen, step;
    uint32_t bsize;
    int lit_off;   // literal compression disabled (fast strategy with targetLength > 0)
};

// clevels.h:25-130 rows 0..2 (W, H, minMatch, targetLength, strategy is fast)
__host__ __device__ inline ZParams params_for(int level, uint64_t n) {
    const uint8_t rows[4][3][5] = {
        {{19, 13, 6, 1, 1}, {19, 14, 7, 0, 1}, {20, 16, 6, 0, 1}},
        {{18, 13, 5, 1, 1}, {18, 14, 6, 0, 1}, {18, 16, 5, 0, 0}},
        {{17, 12, 5, 1, 1}, {17, 13, 6, 0, 1}, {17, 15, 5, 0, 1}},
        {{14, 13, 5, 1, 1}, {14, 15, 5, 0, 1}, {14, 15, 4, 0, 1}},
    };
    ZParams p{};
    const int unknown = n == 0;                               // ZSTD_getParams: 0 = unknown size
    const int tid = unknown ? 0 : (n <= 262144) + (n <= 131072) + (n <= 16384);
    const int row = level < 0 ? 0 : level;
    if (level == 0 || row > 2 || !rows[tid][row][4]) { p.ok = 0; return p; }
    p.ok = 1;
    p.wlog = rows[tid][row][0];
    p.hlog = rows[tid][row][1];
    p.mls = rows[tid][row][2];
    p.tlen = level < 0 ? (uint32_t)(-(level < -131072 ? -131072 : level)) : rows[tid][row][3];
    if (!unknown && n < (1ull << 30)) {                       // ZSTD_adjustCParams_internal
        uint32_t srcLog = 6;
        if (n >= 64) { srcLog = 1; while ((1ull << srcLog) < n) srcLog++; }
        if (p.wlog > srcLog) p.wlog = srcLog;
    }
    if (!unknown && p.hlog > p.wlog + 1) p.hlog = p.wlog + 1;
    if (p.wlog < 10) p.wlog = 10;
    p.step = p.tlen > 1 ? p.tlen + 1 : 2;                     // zstd_fast.c:102, hasStep = targetLength > 1
    p.lit_off = p.tlen > 0;                                    // ZSTD_literalsCompressionIsDisabled
    uint64_t b = 1ull << p.wlog;
    if (b > 131072) b = 131072;
    if (n && b > n) b = n;
    p.bsize = (uint32_t)(b ? b : 1);
    return p;
}

// Per-frame scratch (device memory after the staging slots); layout shared with api.cpp.
struct FrameHdr {            // 64 bytes
    uint32_t ns, nl;         // sequences / literals of the current block (match kernel -> entropy kernel)
    uint32_t nrep0, nrep1;   // repcodes at the end of the current block's parse
    uint32_t rep0, rep1;     // confirmed repcodes (entropy kernel -> next block's parse)
    uint32_t huf_repeat;     // previous Huffman table usable (HUF_repeat_check)
    uint32_t out_off;        // bytes of the frame written to its staging slot
    uint32_t skip;           // block too small to compress (ZSTD_buildSeqStore: raw)
    uint32_t pad[7];
};
constexpr uint32_t kHufOff = 64;                  // prev Huffman table: nb[256] u8 + val[256] u16
constexpr uint32_t kSeqOff = 1024;

struct Layout {
    uint64_t seq_off, lit_off, att_off, tmp_off, tab_off, stride;
};
__host__ __device__ inline Layout layout_for(uint32_t bsize, uint32_t hlog_max) {
    Layout L;
    L.seq_off = kSeqOff;
    L.lit_off = L.seq_off + ((((uint64_t)bsize / 4 + 16) * 8 + 255) & ~255ull);
    L.att_off = L.lit_off + (((uint64_t)bsize + 64 + 255) & ~255ull);      // literals of the block
    L.tmp_off = L.att_off + (((uint64_t)bsize * 4 + 4096 + 255) & ~255ull); // block attempt
    L.tab_off = L.tmp_off + (((uint64_t)bsize + 256 + 255) & ~255ull);      // one Huffman stream
    L.stride = L.tab_off + (4ull << hlog_max);                              // hash table between blocks
    L.stride = (L.stride + 255) & ~255ull;
    return L;
}

// ------------------------------------------------------------------ device helpers
__device__ __forceinline__ uint32_t zhash(uint64_t v, uint32_t hlog, uint32_t mls) {
    switch (mls) {
        case 5: return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - hlog));
        case 6: return (uint32_t)(((v << 16) * 227718039650203ull) >> (64 - hlog));
        case 7: return (uint32_t)(((v << 8) * 58295818150454627ull) >> (64 - hlog));
        default: return ((uint32_t)v * 2654435761u) >> (32 - hlog);
    }
}

#ifdef LZH_ISA_MARKS
#define ZMK(i) asm volatile("; ZMK " #i ::: "memory")
#else
#define ZMK(i) ((void)0)
#endif
// the hash with the minimum match length fixed at compile time (kMls 4..7) or read from P (kMls 0)
template <int kMls>
__device__ __forceinline__ uint32_t zh(uint64_t v, uint32_t hlog, uint32_t mls) { return zhash(v, hlog, kMls ? (uint32_t)kMls : mls); }

// 8 bytes at pos (little endian) from aligned dwords
__device__ __forceinline__ uint64_t ld64(const Bytes& b, int pos) {
    const int X = pos + b.sh, a = X & ~3;
    const uint32_t w0 = ld_b32(b.r, a), w1 = ld_b32(b.r, a + 4), w2 = ld_b32(b.r, a + 8);
    const uint32_t s = (uint32_t)X & 3u;
    const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, s), hi = __builtin_amdgcn_alignbyte(w2, w1, s);
    return (uint64_t)lo | ((uint64_t)hi << 32);
}

struct LdsTab {
    LDSA uint32_t* t;
    __device__ __forceinline__ uint32_t get(uint32_t h) const { return ((volatile LDSA uint32_t*)t)[h]; }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const { ((volatile LDSA uint32_t*)t)[h] = v; }
    __device__ __forceinline__ void claim(uint32_t h, uint32_t v) const { put(h, v); }
    __device__ __forceinline__ uint32_t back(uint32_t h) const { return get(h); }
    static constexpr uint32_t kBackMask = ~0u;
    __device__ __forceinline__ void fence() const { wave_lds_fence(); }
};
// the same table as 16-bit low halves + 8-bit high bytes (3 bytes an entry: 6 waves per CU instead of
// 5 at hashLog 13), for frames below 16 MiB.  A claim writes both halves with the same lanes to the
// same slots, so the hardware's choice among colliding lanes is the same for both stores.
struct LdsTab24 {
    LDSA uint16_t* lo;
    LDSA uint8_t* hi;
    __device__ __forceinline__ uint32_t get(uint32_t h) const {
        return (uint32_t)((volatile LDSA uint16_t*)lo)[h] | ((uint32_t)((volatile LDSA uint8_t*)hi)[h] << 16);
    }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const {
        ((volatile LDSA uint16_t*)lo)[h] = (uint16_t)v;
        ((volatile LDSA uint8_t*)hi)[h] = (uint8_t)(v >> 16);
    }
    __device__ __forceinline__ void claim(uint32_t h, uint32_t v) const { put(h, v); }
    __device__ __forceinline__ uint32_t back(uint32_t h) const { return get(h); }
    static constexpr uint32_t kBackMask = ~0u;
    __device__ __forceinline__ void fence() const { wave_lds_fence(); }
};
// 17-bit entries for frames of at most 128 KiB (positions + 1 < 2^17): 16-bit low halves + a bitmap
// of bit 16 -- 17 KiB at hashLog 13, 9 waves per CU instead of 6.  A put writes the low half and
// clears / sets the bit with LDS atomics (lanes of one bitmap dword touch different bits).  When lanes
// of a batch claim the same slot, the hardware's low-half winner and the bit may come from different
// lanes; such slots are rewritten by a single lane before anything reads them (the batch's restore),
// and a claim's readback compares low halves only (positions of a batch differ by < 2^16).
struct LdsTab17 {
    LDSA uint16_t* lo;
    LDSA uint32_t* bm;
    __device__ __forceinline__ uint32_t get(uint32_t h) const {
        const uint32_t w = ((volatile LDSA uint32_t*)bm)[h >> 5];
        return (uint32_t)((volatile LDSA uint16_t*)lo)[h] | (((w >> (h & 31u)) & 1u) << 16);
    }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const {
        ((volatile LDSA uint16_t*)lo)[h] = (uint16_t)v;
        // bit h & 31 of the bitmap dword := bit 16 of v in one atomic (ds_mskor_b32: M = (M & ~mask) | data)
        const uint32_t a = (uint32_t)(uintptr_t)(bm + (h >> 5));
        asm volatile("ds_mskor_b32 %0, %1, %2" ::"v"(a), "v"(1u << (h & 31u)), "v"(((v >> 16) & 1u) << (h & 31u)) : "memory");
    }
    // the claim writes whole entries (an uncontested slot keeps it); its readback reads the low half
    __device__ __forceinline__ void claim(uint32_t h, uint32_t v) const { put(h, v); }
    __device__ __forceinline__ uint32_t back(uint32_t h) const { return ((volatile LDSA uint16_t*)lo)[h]; }
    static constexpr uint32_t kBackMask = 0xffffu;
    __device__ __forceinline__ void fence() const { wave_lds_fence(); }
};

struct GlbTab {
    rsrc_t r;
    __device__ __forceinline__ uint32_t get(uint32_t h) const {
        return __builtin_amdgcn_raw_buffer_load_b32(r, (int)(h * 4), 0, 1);   // (glc: bypass L1)
    }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const { st_b32(r, (int)(h * 4), v); }
    __device__ __forceinline__ void claim(uint32_t h, uint32_t v) const { put(h, v); }
    __device__ __forceinline__ uint32_t back(uint32_t h) const { return get(h); }
    static constexpr uint32_t kBackMask = ~0u;
    __device__ __forceinline__ void fence() const { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
};

// number of equal bytes at a and b (a < b never required), at most maxn; wave-parallel, 256 bytes a round
__device__ int count_fwd(const Bytes& in, int a, int b, int maxn, int lane) {
    int n = 0;
    while (n < maxn) {
        const int off = n + 4 * lane;
        uint32_t first = 64 * 4;
        if (off < maxn) {
            const uint32_t x = ld_u32(in.r, a + off + in.sh) ^ ld_u32(in.r, b + off + in.sh);
            int eq = x ? (int)(__builtin_ctz(x) >> 3) : 4;
            if (off + eq > maxn) eq = maxn - off;
            if (eq < 4) first = (uint32_t)(4 * lane + eq);
        }
        const uint64_t m = ballot(first < 256u);
        if (m) return n + (int)rdlane(first, ffs64(m));
        n += 256;
    }
    return maxn;
}

// bytes equal going backwards from a-1 / b-1, at most maxn
__device__ int count_bwd(const Bytes& in, int a, int b, int maxn, int lane) {
    int n = 0;
    while (n < maxn) {
        const int k = n + lane;
        const bool stop = k >= maxn || in.b(a - 1 - k) != in.b(b - 1 - k);
        const uint64_t m = ballot(stop);
        if (m) return n + ffs64(m);
        n += 64;
    }
    return maxn;
}

struct SeqOut {
    rsrc_t seq;      // u64 per sequence: ll (20 bits) | ml (20 bits) << 20 | offBase << 40
    Bytes lits;
    int ns, nl;
    __device__ __forceinline__ void put(int lane, uint32_t ll, uint32_t off, uint32_t ml) {
        if (lane == 0) {
            const uint64_t v = (uint64_t)ll | ((uint64_t)ml << 20) | ((uint64_t)off << 40);
            st_b32(seq, ns * 8, (uint32_t)v);
            st_b32(seq, ns * 8 + 4, (uint32_t)(v >> 32));
        }
        ns++;
    }
};

__device__ __forceinline__ void pair_step(int& A, int& D, int& s, int& nx) {
    A += D;
    D = s;
    if (A + s >= nx) { s++; nx += 128; }
}

template <int kMls = 0, class Tab>
__device__ void tab_put_pos(const Tab& T, const Bytes& in, int pos, const ZParams& P) {
    const uint32_t h = zh<kMls>(ld64(in, pos), P.hlog, P.mls);
    T.put(h, (uint32_t)pos + 1);
}

#ifndef LZH_ZSTDC_STATS
#define LZH_ZSTDC_STATS 0   // match / entropy kernel phase clocks (tools/zstdc_stats.py)
#endif
#if LZH_ZSTDC_STATS
__device__ unsigned long long lzh_zstdc_stats_buf[24];
#endif
// match-kernel phase clocks (indices 0..5: search batches, match, fills + repcodes, batches, sequences,
// frames), accumulated in registers and added once per frame
struct MStat {
    uint64_t v[5] = {0, 0, 0, 0, 0}, last = 0;
    __device__ __forceinline__ void mark(int i) {
        if (LZH_ZSTDC_STATS) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            v[i] += t - last;
            last = t;
        }
    }
    __device__ __forceinline__ void start() { if (LZH_ZSTDC_STATS) last = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void count(int i) { if (LZH_ZSTDC_STATS) v[i]++; }
    __device__ __forceinline__ void flush(int lane) {
#if LZH_ZSTDC_STATS
        if (lane == 0) {
            for (int i = 0; i < 5; i++) atomicAdd(&lzh_zstdc_stats_buf[i], (unsigned long long)v[i]);
            atomicAdd(&lzh_zstdc_stats_buf[5], 1ull);
        }
#endif
    }
};

// The parse of one block [bs, be) of a frame (positions relative to the frame start; table
// entries hold position + 1, 0 = empty).  Mirrors zstd_fast.c:92-315.
// dst[d0, d0+len) = src[s0, s0+len) for one wave: runs of up to 256 bytes load everything first
// (head bytes, one dword per lane, tail bytes; positions clamped, nothing predicated) and store after
// one wait; longer runs take copy_span
#ifndef LZH_ZSTD_LITB
#define LZH_ZSTD_LITB 64   // literal runs up to this many bytes: one byte per lane (no head / dword / tail split)
#endif
__device__ __forceinline__ void lit_copy(const Bytes& src, int s0, const Bytes& dst, int d0, int len, int lane) {
    if (len <= 0) return;
    if (len <= LZH_ZSTD_LITB) {
        const bool on = lane < len;
        const uint32_t v = src.b(s0 + (on ? lane : 0));
        if (on) dst.st8(d0 + lane, v);
        return;
    }
    if (len > 4 * LZH_WAVE) { copy_span(src, s0, dst, d0, len, lane, LZH_WAVE); return; }
    const int head = min(len, (4 - ((d0 + dst.sh) & 3)) & 3);
    const int nd = (len - head) >> 2, t0 = head + 4 * nd;
    const bool hl = lane < head, dl = lane < nd, tl = lane < len - t0;
    const uint32_t hb = src.b(s0 + (hl ? lane : 0));
    const uint32_t w = src.w32(s0 + (dl ? head + 4 * lane : 0));
    const uint32_t tb = src.b(s0 + (tl ? t0 + lane : 0));
    if (hl) dst.st8(d0 + lane, hb);
    if (dl) dst.st32_aligned(d0 + head + 4 * lane, w);
    if (tl) dst.st8(d0 + t0 + lane, tb);
}

#ifndef LZH_ZSTD_PREF
#define LZH_ZSTD_PREF 1   // the first batch's loads issued with the previous sequence's table fills
#endif
#ifndef LZH_ZSTD_FWD
#define LZH_ZSTD_FWD 16   // lanes of the forward compare in the match's round trip (4 bytes each; longer: count_fwd)
#endif
#ifndef LZH_ZSTD_BWD
#define LZH_ZSTD_BWD 16   // lanes of the backward compare in the match's round trip (1 byte each; longer: count_bwd)
#endif
template <int kMls = 0, class Tab>
__device__ void fast_block(const Tab& T, const Bytes& in, const ZParams& P, int bs, int be, uint32_t rep[2],
                           SeqOut& O, int lane) {
    const int W = 1 << P.wlog;
    const int dl = bs > W ? bs - W : 0;                     // ZSTD_window_enforceMaxDist at the block start
    const int pstart = (be - dl > W) ? be - W : dl;        // ZSTD_getLowestPrefixIndex(blockEnd)
    const int ilimit = be - 8;
    int ip = bs + (bs == pstart);
    int anchor = bs;
    uint32_t r1 = rep[0], r2 = rep[1], saved = 0;
    {
        const int wlow = (ip - dl > W) ? ip - W : dl;
        const uint32_t maxRep = (uint32_t)(ip - wlow);
        if (r2 > maxRep) { saved = r2; r2 = 0; }
        if (r1 > maxRep) { saved = r1; r1 = 0; }
    }
    const int j = lane >> 1, half = lane & 1;
    const uint64_t below = (1ull << lane) - 1ull;
    MStat ms;
    ms.start();
    // probe schedule of a batch from (A, D, s, nx): pair j of lane (A_j, D_j), and the state after 32 pairs
    struct Sched { int Aj, Dj, A32, D32, s32, n32; };
    auto sched = [&](int A, int D, int s, int nx) -> Sched {
        Sched S;
        if (D == 2 && s == 2 && A + 62 < nx) {
            S.Aj = A + 2 * j;
            S.Dj = 2;
            S.A32 = A + 60; S.D32 = 2; S.s32 = 2; S.n32 = nx;
            pair_step(S.A32, S.D32, S.s32, S.n32);
            pair_step(S.A32, S.D32, S.s32, S.n32);
        } else {
            int a = A, d = D, ss = s, nn = nx;
            for (int i = 0; i < j; i++) pair_step(a, d, ss, nn);
            S.Aj = a;
            S.Dj = d;
            pair_step(a, d, ss, nn);
            S.A32 = rdlanei(a, 63); S.D32 = rdlanei(d, 63); S.s32 = rdlanei(ss, 63); S.n32 = rdlanei(nn, 63);
        }
        return S;
    };
    // a batch's P-side and rep-side loads (branch-free: clamped positions)
    struct PLoad { uint64_t w8; uint32_t rv, rm; };
    auto pload = [&](const Sched& S, int A) -> PLoad {
        const bool valid = j == 0 || S.Aj + 1 + S.Dj < ilimit;
        const bool rok = valid && !half && r1 > 0;
        PLoad L;
        L.w8 = ld64(in, valid ? S.Aj + half : A);
        L.rv = in.w32(rok ? S.Aj + S.Dj : A);
        L.rm = in.w32(rok ? S.Aj + S.Dj - (int)r1 : A);
        return L;
    };
    // the first batch after a sequence is scheduled and loaded with that sequence's table fills (one
    // round trip for both); a repcode sequence there moves the start and drops it
    bool pre = false;
    Sched S0{};
    PLoad L0{};
    for (;;) {
        if (ip + (int)P.step + 1 >= ilimit) break;
        int A = ip, D = (int)P.step, s = (int)P.step, nx = ip + 128;
        int kind = 0, ev = 0, ecand = 0;
        int eA = 0, eD = 0;
        bool ended = false;
        Sched S;
        PLoad Ld;
        if (LZH_ZSTD_PREF && pre) {
            S = S0;
            Ld = L0;
        } else {
            S = sched(A, D, s, nx);
            Ld = pload(S, A);
        }
        for (;;) {
            ZMK(0);
            ms.count(3);
            const int Aj = S.Aj, Dj = S.Dj, A32 = S.A32, D32 = S.D32, s32 = S.s32, n32 = S.n32;
            const bool valid = j == 0 || Aj + 1 + Dj < ilimit;
            const uint64_t vmask = ballot(Aj + 1 + Dj < ilimit) | 3ull;   // (pair 0 = lanes 0, 1: one compare)
            const int q = Aj + half;
            ZMK(1);
            // ---- P side, rep side
            const uint64_t w8 = Ld.w8;
            const uint32_t rv = Ld.rv, rm = Ld.rm;
            const uint32_t h = zh<kMls>(w8, P.hlog, P.mls);
            ZMK(2);
            // ---- table read, claim, read back
            uint32_t old = 0, back = 0;
            if (valid) old = T.get(h);
            // the compare load for the slot's old value goes out before the claim round trip (a lane
            // whose slot an earlier lane of the batch claimed compares against that lane's bytes)
            const bool ook = valid && old > (uint32_t)pstart;
            const uint32_t cwo = in.w32(ook ? (int)old - 1 : A);
            T.fence();
            if (valid) T.claim(h, (uint32_t)q + 1);
            T.fence();
            if (valid) back = T.back(h);
            const uint64_t losers = ballot(back != (((uint32_t)q + 1) & Tab::kBackMask)) & vmask;
            uint64_t grp = 1ull << lane;
            int prev = -1;
            if (losers) {
                // lanes of one slot read back the same winner: group by equal winner (bit-sliced over
                // the winner's offset from the batch's first position)
                const int A0 = rdlanei(Aj, 0);
                const int span = rdlanei(Aj, 62) + 2 - A0;
                const int nbits = span > 2 ? 32 - __builtin_clz((uint32_t)span - 1u) : 1;   // ceil(log2 span), >= 1
                const uint32_t wr = (back - 1u - (uint32_t)A0) & Tab::kBackMask;
                uint64_t eq = vmask;
                // (the first 6 bits unrolled, without the loop's scalar chain: bits at or past nbits are 0
                // in every valid lane's offset, so those rounds leave eq as it is)
                // (ballot of the single compare, masked with vmask in scalar: a ballot of a compound condition goes
                // through a VGPR and back)
#pragma unroll
                for (int b = 0; b < 6; b++) {
                    const bool wb = (wr >> b) & 1u;
                    const uint64_t bm = ballot(wb) & vmask;
                    eq &= wb ? bm : ~bm;
                }
                for (int b = 6; b < nbits; b++) {
                    const bool wb = (wr >> b) & 1u;
                    const uint64_t bm = ballot(wb) & vmask;
                    eq &= wb ? bm : ~bm;
                }
                grp = valid ? eq : grp;
                const uint64_t eb = grp & below;
                prev = (valid && eb) ? 63 - __builtin_clzll(eb) : -1;
            }
            uint32_t cand = old;
            // (hits as lane masks from single compares: a ballot of a compound or merged condition goes through
            // a VGPR and back)
            uint64_t H = ballot(cwo == (uint32_t)w8) & ballot(old > (uint32_t)pstart) & vmask;
            if (losers) {   // (a batch without a collision needs no gathers: most batches)
                const int src = prev < 0 ? lane : prev;
                const int qprev = lane_gather((uint32_t)q, src);
                const uint32_t wprev = lane_gather((uint32_t)w8, src);
                if (prev >= 0) cand = (uint32_t)qprev + 1;
                const uint64_t PV = ballot(prev >= 0);              // colliders (valid lanes only)
                H = (H & ~PV) | (ballot(wprev == (uint32_t)w8) & PV);
            }
            ZMK(3);
            // ---- candidate compare (an in-batch candidate is past the prefix start)
            // (R: the compare's ballot masked in scalar -- rok is vmask, even lanes, r1 > 0)
            const uint64_t R = r1 > 0 ? ballot(rv == rm) & vmask & 0x5555555555555555ull : 0ull;
            const uint64_t E = R | H;
            ZMK(4);
            const uint64_t committed = E ? (vmask & (ffs64(E) == 63 ? ~0ull : ((2ull << ffs64(E)) - 1ull))) : vmask;
            // ---- slots: the value the sequential order leaves (no collision in the batch: each lane
            // owns its slot, and the lanes past the first event put the old value back)
            if (!losers) {
                if (valid && !lane_on(committed)) T.put(h, old);
            } else if (valid) {
                const uint64_t gc = grp & committed;
                bool writer;
                uint32_t val;
                if (gc) { writer = lane == 63 - __builtin_clzll(gc); val = (uint32_t)q + 1; }
                else { writer = lane == ffs64(grp); val = old; }
                if (writer && (losers || !gc)) T.put(h, val);
            }
            T.fence();
            if (E) {
                ev = ffs64(E);
                kind = (ev & 1) ? 3 : (((R >> ev) & 1ull) ? 1 : 2);
                eA = rdlanei(Aj, ev);
                eD = rdlanei(Dj, ev);
                ecand = (int)rdlane(cand, ev);
                break;
            }
            if (vmask != ~0ull || A32 + 1 + D32 >= ilimit) { ended = true; break; }
            A = A32; D = D32; s = s32; nx = n32;
            S = sched(A, D, s, nx);
            Ld = pload(S, A);
        }
        ms.mark(0);
        if (ended) break;
        ZMK(5);
        ms.count(4);
        // ---- the match.  m0 / p0: its start and source before the backward extension; the bytes
        // of the backward and forward compares and the literal run [anchor, m0) are loaded in one
        // round trip (the forward count from m0 + 4 does not depend on the backward extension; the
        // literal copy writes past the final literal count when it extends, and the next run
        // overwrites those bytes)
        int m0, p0, bmax, cur0, ip1;
        uint32_t offBase;
        if (kind == 1) {
            m0 = eA + eD;
            p0 = m0 - (int)r1;
            bmax = 1;                                     // ip0[-1] == match0[-1], zstd_fast.c:204-211
            offBase = 1;
            cur0 = eA;
            ip1 = eA + 1;
        } else {
            m0 = kind == 2 ? eA : eA + 1;
            p0 = ecand - 1;
            r2 = r1;
            r1 = (uint32_t)(m0 - p0);
            offBase = r1 + 3;
            cur0 = m0;
            ip1 = kind == 2 ? eA + 1 : eA + eD;
            bmax = max(0, min(m0 - anchor, p0 - pstart));
        }
        const int fmax = be - (m0 + 4);
        const bool bl = lane < bmax && lane < LZH_ZSTD_BWD, fl = lane < LZH_ZSTD_FWD && 4 * lane < fmax;
        // (every load unconditional at a clamped position, literal loads included: one wait for all --
        // loads under lane-divergent branches each got their own wait inside the branch)
        const uint32_t ba = in.b(bl ? m0 - 1 - lane : m0), bb = in.b(bl ? p0 - 1 - lane : m0);
        const uint32_t fa = ld_u32(in.r, (fl ? m0 + 4 + 4 * lane : m0) + in.sh),
                       fb = ld_u32(in.r, (fl ? p0 + 4 + 4 * lane : m0) + in.sh);
        lit_copy(in, anchor, O.lits, O.nl, m0 - anchor, lane);
        int bk;
        {
            constexpr int kB = LZH_ZSTD_BWD;
            const int nbl = min(bmax, LZH_ZSTD_BWD);               // (the lanes of bl, as a scalar mask)
            const uint64_t m = ~(nbl >= 64 ? ~0ull : (1ull << max(nbl, 0)) - 1ull) | ballot(ba != bb);
            bk = ffs64(m);
            if (bk >= kB && bmax > kB) bk = kB + count_bwd(in, m0 - kB, p0 - kB, bmax - kB, lane);
            bk = min(bk, bmax);
        }
        int fw;
        {
            const uint32_t x = fa ^ fb;
            int eq = x ? (int)(__builtin_ctz(x) >> 3) : 4;
            if (4 * lane + eq > fmax) eq = fmax - 4 * lane;
            const int nfl = min(LZH_ZSTD_FWD, fmax > 0 ? (fmax + 3) >> 2 : 0);   // (the lanes of fl)
            const uint64_t m = ballot(eq < 4) & (nfl >= 64 ? ~0ull : (1ull << nfl) - 1ull);
            constexpr int kF = 4 * LZH_ZSTD_FWD;
            if (m) fw = 4 * ffs64(m) + (int)rdlane((uint32_t)eq, ffs64(m));
            else fw = fmax <= kF ? max(fmax, 0) : kF + count_fwd(in, m0 + 4 + kF, p0 + 4 + kF, fmax - kF, lane);
        }
        ZMK(6);
        ms.mark(1);
        const int mstart = m0 - bk;
        const int len = 4 + bk + fw;
        O.nl += mstart - anchor;
        O.put(lane, (uint32_t)(mstart - anchor), offBase, (uint32_t)len);
        ip = mstart + len;
        anchor = ip;
        {   // table fills (zstd_fast.c:216-231) and the immediate repcode check: loads in one round trip
            const uint64_t h1 = ld64(in, ip1), h2 = ld64(in, cur0 + 2), h3 = ld64(in, ip - 2);
            const uint32_t c0 = in.w32(ip), c1 = in.w32(ip - (int)r2);
            if (LZH_ZSTD_PREF) {   // (unconditional: past ilimit the loop ends and they go unused)
                S0 = sched(ip, (int)P.step, (int)P.step, ip + 128);
                L0 = pload(S0, ip);
                pre = true;
            }
            if (lane == 0) {
                if (ip1 < ip) T.put(zh<kMls>(h1, P.hlog, P.mls), (uint32_t)ip1 + 1);
                if (ip <= ilimit) {
                    T.put(zh<kMls>(h2, P.hlog, P.mls), (uint32_t)cur0 + 3);
                    T.put(zh<kMls>(h3, P.hlog, P.mls), (uint32_t)ip - 1);
                }
            }
            T.fence();
            bool more = ip <= ilimit && r2 > 0 && c0 == c1;
            while (more) {
                pre = false;
                const int rl = 4 + count_fwd(in, ip + 4, ip + 4 - (int)r2, be - (ip + 4), lane);
                const uint32_t t = r2; r2 = r1; r1 = t;
                if (lane == 0) tab_put_pos<kMls>(T, in, ip, P);
                T.fence();
                O.put(lane, 0, 1, (uint32_t)rl);
                ip += rl;
                anchor = ip;
                more = ip <= ilimit && r2 > 0 && in.w32(ip) == in.w32(ip - (int)r2);
            }
        }
        ms.mark(2);
    }
    ms.flush(lane);
    rep[0] = r1 ? r1 : saved;
    rep[1] = r2 ? r2 : saved;
    copy_span(in, anchor, O.lits, O.nl, be - anchor, lane, LZH_WAVE);   // last literals
    O.nl += be - anchor;
}

#ifndef LZH_ZSTD_TAB17
#define LZH_ZSTD_TAB17 1   // 17-bit hash-table entries (LdsTab17) for chunks <= 128 KiB
#endif

#if LZH_ZSTDC_STATS
// entropy-kernel phase clocks (indices 16..23): lane 0 adds the clocks since its previous mark
#define ZEM(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); if (threadIdx.x == 0) atomicAdd(&lzh_zstdc_stats_buf[16 + (i)], (unsigned long long)(t_ - ze_last)); ze_last = t_; } while (0)
#define ZEM_DECL uint64_t ze_last = __builtin_amdgcn_s_memtime()
#else
#define ZEM(i) ((void)0)
#define ZEM_DECL ((void)0)
#endif

}  // namespace zc

using namespace zc;

// one wave per frame; block k of every frame
extern "C" __global__ void __launch_bounds__(64)
lzh_zstd_match_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size, int level,
                      int k, uint8_t* scratch, uint64_t fstride, uint64_t seq_off, uint64_t lit_off, uint64_t tab_off,
                      uint32_t lds_arg, uint32_t f0) {
    extern __shared__ __attribute__((aligned(16))) uint32_t zlds[];
    const int lane = threadIdx.x;
    const uint64_t f = (uint64_t)blockIdx.x + f0;   // (f0: the launch's first frame)
    const uint64_t ioff = f * chunk_size;
    if (ioff >= n_total && !(n_total == 0 && f == 0)) return;
    const uint64_t nf = n_total ? min(chunk_size, n_total - ioff) : 0;
    const ZParams P = params_for(level, nf);
    if (!P.ok) return;
    const uint64_t nblocks = nf ? (nf + P.bsize - 1) / P.bsize : 1;
    if ((uint64_t)k >= nblocks) return;
    uint8_t* fs = scratch + f * fstride;
    rsrc_t hdr = make_rsrc(fs, 64);
    const int bs = k * (int)P.bsize;
    const int be = (int)min<uint64_t>(nf, (uint64_t)bs + P.bsize);
    if (be - bs < 7) {                                   // ZSTD_buildSeqStore: too small, stored raw
        if (lane == 0) { st_b32(hdr, 32, 1u); st_b32(hdr, 0, 0u); st_b32(hdr, 4, 0u); }
        return;
    }
    Bytes in_b;
    in_b.init(in + ioff, min<uint64_t>(in_readable - ioff, nf + 16));
    SeqOut O;
    O.seq = make_rsrc(fs + seq_off, (uint32_t)(lit_off - seq_off));
    O.lits.init(fs + lit_off, P.bsize + 64);
    O.ns = 0;
    O.nl = 0;
    uint32_t rep[2] = {1u, 4u};                          // repStartValue
    if (k > 0) { rep[0] = uni(ld_b32(hdr, 16)); rep[1] = uni(ld_b32(hdr, 20)); }
    const uint32_t tbytes = 4u << P.hlog;
    const uint32_t nent = 1u << P.hlog;
    const uint32_t lds_table_bytes = lds_arg;          // the table's bytes in dynamic LDS (0: global)
    const uint32_t bmb = max(nent / 8u, 4u);            // LdsTab17 bitmap bytes
    if (LZH_ZSTD_TAB17 && chunk_size <= 131072u && nblocks == 1 && 2u * nent + bmb <= lds_table_bytes) {
        // (single-block frames: the table starts empty and is not saved)
        LdsTab17 T{(LDSA uint16_t*)zlds, (LDSA uint32_t*)((LDSA uint8_t*)zlds + 2 * nent)};
        for (uint32_t i = lane; i < (2u * nent + bmb) / 4u; i += 64) ((volatile LDSA uint32_t*)zlds)[i] = 0u;
        T.fence();
        if (P.mls == 6) fast_block<6>(T, in_b, P, bs, be, rep, O, lane);   // (hash fixed at compile time)
        else if (P.mls == 5) fast_block<5>(T, in_b, P, bs, be, rep, O, lane);
        else fast_block(T, in_b, P, bs, be, rep, O, lane);
    } else if (chunk_size < (16u << 20) && 3u * nent <= lds_table_bytes) {
        LdsTab24 T{(LDSA uint16_t*)zlds, (LDSA uint8_t*)zlds + 2 * nent};
        rsrc_t save = make_rsrc(fs + tab_off, tbytes);
        for (uint32_t i = lane; i < nent; i += 64) T.put(i, k == 0 ? 0u : ld_b32(save, (int)(i * 4)));
        T.fence();
        fast_block(T, in_b, P, bs, be, rep, O, lane);
        if ((uint64_t)k + 1 < nblocks)
            for (uint32_t i = lane; i < nent; i += 64) st_b32(save, (int)(i * 4), T.get(i));
    } else if (tbytes <= lds_table_bytes) {
        LdsTab T{(LDSA uint32_t*)zlds};
        rsrc_t save = make_rsrc(fs + tab_off, tbytes);
        for (uint32_t i = lane; i < tbytes / 4; i += 64) T.put(i, k == 0 ? 0u : ld_b32(save, (int)(i * 4)));
        T.fence();
        fast_block(T, in_b, P, bs, be, rep, O, lane);
        if ((uint64_t)k + 1 < nblocks)
            for (uint32_t i = lane; i < tbytes / 4; i += 64) st_b32(save, (int)(i * 4), T.get(i));
    } else {
        GlbTab T{make_rsrc(fs + tab_off, tbytes)};
        if (k == 0) {
            for (uint32_t i = lane; i < tbytes / 4; i += 64) T.put(i, 0u);
            T.fence();
        }
        fast_block(T, in_b, P, bs, be, rep, O, lane);
    }
    if (lane == 0) {
        st_b32(hdr, 0, (uint32_t)O.ns);
        st_b32(hdr, 4, (uint32_t)O.nl);
        st_b32(hdr, 8, rep[0]);
        st_b32(hdr, 12, rep[1]);
        st_b32(hdr, 32, 0u);
    }
}

// ======================================================================= entropy stage
namespace ze {

typedef int16_t s16;

struct HNode { uint32_t count; uint16_t parent; uint8_t byte; uint8_t nb; };

struct Fse {                    // FSE compression table (FSE_buildCTable_wksp layout, split)
    uint16_t st[512];
    int32_t dfs[64];
    uint32_t dnb[64];
    uint32_t tlog;
};

struct Lds {
    uint32_t cnt3[3][64];       // LL / OF / ML code histograms
    // the Huffman tree while the literals' table is built (huf_build), the FSE tables after it: the
    // weights' table (fse[0], huf_compress_weights) and the sequences' tables
    union {
        HNode node[514];
        Fse fse[3];
    };
    uint8_t nb[256];            // fresh Huffman table
    uint16_t val[256];
    uint8_t pnb[256];           // previous block's Huffman table (frame scratch)
    uint16_t pval[256];
    s16 norm[64];
    // the literals section's workspace, then the sequences section's (the two unions: 13 waves per CU
    // instead of 8)
    union {
        struct {
            uint32_t cnt[256];  // literal histogram
            uint8_t w[256];     // Huffman weights
            uint8_t hdr[264];   // Huffman table header
            int32_t qs[2 * 300];   // quick-sort task stack (the sequence encoder's table deltas later)
        };
        struct {
            uint8_t symAt[512];    // FSE spread workspace
            uint32_t cumul[64];
            uint32_t sq[64 * 3];   // a group's (nbBits << 16 | bits) per state chain
        };
    };
    uint32_t stage[192];        // bit staging window (64 sequences of <= 90 bits)
    uint32_t misc[16];
};

__device__ __forceinline__ uint32_t hb32(uint32_t v) { return 31u - (uint32_t)__builtin_clz(v); }

__device__ __forceinline__ uint32_t ll_code(uint32_t ll) {
    if (ll < 16) return ll;
    if (ll < 64) {
        if (ll < 24) return 16 + ((ll - 16) >> 1);
        if (ll < 32) return 20 + ((ll - 24) >> 2);
        if (ll < 48) return 22 + ((ll - 32) >> 3);
        return 24;
    }
    return hb32(ll) + 19;
}
__device__ __forceinline__ uint32_t ml_code(uint32_t mb) {
    if (mb < 32) return mb;
    if (mb < 128) {
        if (mb < 40) return 32 + ((mb - 32) >> 1);
        if (mb < 48) return 36 + ((mb - 40) >> 2);
        if (mb < 64) return 38 + ((mb - 48) >> 3);
        if (mb < 96) return 40 + ((mb - 64) >> 4);
        return 42;
    }
    return hb32(mb) + 36;
}
// extra bits of a literal-length / match-length code (kLLB / kMLB below) from the length itself: the
// single-lane sequence encoder runs under lane 0, where a table lookup would be a vector load from
// constant memory (a memory round trip per lookup) instead of a scalar one
__device__ __forceinline__ uint32_t ll_bits(uint32_t ll) {
    return ll < 16 ? 0u : ll < 24 ? 1u : ll < 32 ? 2u : ll < 48 ? 3u : ll < 64 ? 4u : (uint32_t)hb32(ll);
}
__device__ __forceinline__ uint32_t ml_bits(uint32_t mb) {
    return mb < 32 ? 0u : mb < 40 ? 1u : mb < 48 ? 2u : mb < 64 ? 3u : mb < 96 ? 4u : mb < 128 ? 5u : (uint32_t)hb32(mb);
}
__device__ __constant__ uint8_t kLLB[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3,
                                            4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__device__ __constant__ uint8_t kMLB[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                            0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__device__ __constant__ int16_t kLLDef[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                              2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__device__ __constant__ int16_t kMLDef[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                              1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__device__ __constant__ int16_t kOFDef[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                              -1, -1, -1, -1, -1};

// ---- single-lane byte sinks: global (Bytes) or LDS, and a 64-bit bit accumulator (LSB first)
struct LdsSink {
    LDSA uint8_t* p;
    __device__ __forceinline__ void st8(int pos, uint32_t v) const { p[pos] = (uint8_t)v; }
};
template <class Sink>
struct BitW {
    Sink o;
    int pos;
    uint64_t acc;
    uint32_t nb;
    __device__ __forceinline__ void add(uint64_t v, uint32_t n) {
        if (!n) return;
        v &= (n >= 64) ? ~0ull : ((1ull << n) - 1ull);
        acc |= v << nb;
        nb += n;
        while (nb >= 8) { o.st8(pos++, (uint32_t)acc & 0xffu); acc >>= 8; nb -= 8; }
    }
    __device__ __forceinline__ int close() {
        add(1, 1);
        if (nb) { o.st8(pos++, (uint32_t)acc & 0xffu); acc = 0; nb = 0; }
        return pos;
    }
};

// ---- FSE (fse_compress.c), lane 0 only
__device__ uint32_t fse_min_log(uint32_t n, uint32_t maxs) {
    const uint32_t a = hb32(n) + 1, b = hb32(maxs) + 2;
    return a < b ? a : b;
}
__device__ uint32_t fse_opt_log(uint32_t maxLog, uint32_t n, uint32_t maxs, uint32_t minus) {
    const uint32_t srcBits = hb32(n - 1) - minus;
    uint32_t tl = maxLog ? maxLog : 11;
    const uint32_t mb = fse_min_log(n, maxs);
    if (srcBits < tl) tl = srcBits;
    if (mb > tl) tl = mb;
    if (tl < 5) tl = 5;
    if (tl > 12) tl = 12;
    return tl;
}
__device__ int fse_norm_m2(LDSA s16* norm, uint32_t tl, const LDSA uint32_t* cnt, uint32_t total, uint32_t maxs,
                           s16 low) {
    const s16 NA = -2;
    uint32_t distributed = 0;
    const uint32_t lowThreshold = total >> tl;
    uint32_t lowOne = (uint32_t)(((uint64_t)total * 3) >> (tl + 1));
    for (uint32_t s = 0; s <= maxs; s++) {
        if (cnt[s] == 0) { norm[s] = 0; continue; }
        if (cnt[s] <= lowThreshold) { norm[s] = low; distributed++; total -= cnt[s]; continue; }
        if (cnt[s] <= lowOne) { norm[s] = 1; distributed++; total -= cnt[s]; continue; }
        norm[s] = NA;
    }
    uint32_t toDist = (1u << tl) - distributed;
    if (toDist == 0) return 0;
    if ((total / toDist) > lowOne) {
        lowOne = (uint32_t)(((uint64_t)total * 3) / (toDist * 2));
        for (uint32_t s = 0; s <= maxs; s++)
            if (norm[s] == NA && cnt[s] <= lowOne) { norm[s] = 1; distributed++; total -= cnt[s]; }
        toDist = (1u << tl) - distributed;
    }
    if (distributed == maxs + 1) {
        uint32_t mv = 0, mc = 0;
        for (uint32_t s = 0; s <= maxs; s++) if (cnt[s] > mc) { mv = s; mc = cnt[s]; }
        norm[mv] += (s16)toDist;
        return 0;
    }
    if (total == 0) {
        for (uint32_t s = 0; toDist > 0; s = (s + 1) % (maxs + 1))
            if (norm[s] > 0) { toDist--; norm[s]++; }
        return 0;
    }
    const uint64_t vlog = 62 - tl;
    const uint64_t mid = (1ull << (vlog - 1)) - 1;
    const uint64_t rstep = (((1ull << vlog) * toDist) + mid) / total;
    uint64_t acc = mid;
    for (uint32_t s = 0; s <= maxs; s++) {
        if (norm[s] == NA) {
            const uint64_t end = acc + cnt[s] * rstep;
            const uint32_t w = (uint32_t)(end >> vlog) - (uint32_t)(acc >> vlog);
            if (w < 1) return -1;
            norm[s] = (s16)w;
            acc = end;
        }
    }
    return 0;
}
__device__ int fse_normalize(LDSA s16* norm, uint32_t tl, const LDSA uint32_t* cnt, uint32_t total, uint32_t maxs,
                             int useLow) {
    const uint32_t rtb[8] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};
    if (tl < fse_min_log(total, maxs)) return -1;
    const s16 low = useLow ? -1 : 1;
    const uint64_t scale = 62 - tl;
    const uint64_t step = (1ull << 62) / total;
    const uint64_t vstep = 1ull << (scale - 20);
    int still = 1 << tl;
    uint32_t largest = 0;
    s16 largestP = 0;
    const uint32_t lowThreshold = total >> tl;
    for (uint32_t s = 0; s <= maxs; s++) {
        if (cnt[s] == total) return 0;
        if (cnt[s] == 0) { norm[s] = 0; continue; }
        if (cnt[s] <= lowThreshold) { norm[s] = low; still--; continue; }
        s16 p = (s16)((cnt[s] * step) >> scale);
        if (p < 8) {
            const uint64_t rest = vstep * rtb[p];
            p += (s16)((cnt[s] * step) - ((uint64_t)p << scale) > rest);
        }
        if (p > largestP) { largestP = p; largest = s; }
        norm[s] = p;
        still -= p;
    }
    if (-still >= (norm[largest] >> 1)) return fse_norm_m2(norm, tl, cnt, total, maxs, low);
    norm[largest] += (s16)still;
    return 0;
}
// FSE_writeNCount through a single-lane byte sink at pos; returns bytes written
template <class Sink>
__device__ int fse_write_ncount(const Sink& o, int pos, const LDSA s16* norm, uint32_t maxs, uint32_t tl) {
    const int p0 = pos;
    const int tsize = 1 << tl;
    uint32_t bits = (tl - 5);
    int nb = 4;
    int remaining = tsize + 1, threshold = tsize, nbBits = (int)tl + 1;
    uint32_t sym = 0;
    const uint32_t alpha = maxs + 1;
    int prev0 = 0;
    while (sym < alpha && remaining > 1) {
        if (prev0) {
            uint32_t start = sym;
            while (sym < alpha && !norm[sym]) sym++;
            if (sym == alpha) break;
            while (sym >= start + 24) {
                start += 24;
                bits += 0xFFFFu << nb;
                o.st8(pos, bits & 0xffu); o.st8(pos + 1, (bits >> 8) & 0xffu); pos += 2;
                bits >>= 16;
            }
            while (sym >= start + 3) { start += 3; bits += 3u << nb; nb += 2; }
            bits += (sym - start) << nb;
            nb += 2;
            if (nb > 16) { o.st8(pos, bits & 0xffu); o.st8(pos + 1, (bits >> 8) & 0xffu); pos += 2; bits >>= 16; nb -= 16; }
        }
        {
            int c = norm[sym++];
            const int mx = (2 * threshold - 1) - remaining;
            remaining -= c < 0 ? -c : c;
            c++;
            if (c >= threshold) c += mx;
            bits += (uint32_t)c << nb;
            nb += nbBits;
            nb -= (c < mx);
            prev0 = (c == 1);
            while (remaining < threshold) { nbBits--; threshold >>= 1; }
        }
        if (nb > 16) { o.st8(pos, bits & 0xffu); o.st8(pos + 1, (bits >> 8) & 0xffu); pos += 2; bits >>= 16; nb -= 16; }
    }
    o.st8(pos, bits & 0xffu);
    o.st8(pos + 1, (bits >> 8) & 0xffu);
    pos += (nb + 7) / 8;
    return pos - p0;
}
__device__ void fse_build(LDSA Fse& ct, const LDSA s16* norm, uint32_t maxs, uint32_t tl, LDSA uint8_t* symAt,
                          LDSA uint32_t* cumul) {
    const uint32_t tsize = 1u << tl, mask = tsize - 1, step = (tsize >> 1) + (tsize >> 3) + 3;
    uint32_t high = tsize - 1;
    ct.tlog = tl;
    cumul[0] = 0;
    for (uint32_t u = 1; u <= maxs + 1; u++) {
        if (norm[u - 1] == -1) { cumul[u] = cumul[u - 1] + 1; symAt[high--] = (uint8_t)(u - 1); }
        else cumul[u] = cumul[u - 1] + (uint32_t)norm[u - 1];
    }
    uint32_t pos = 0;
    for (uint32_t s = 0; s <= maxs; s++)
        for (int kk = 0; kk < norm[s]; kk++) {
            symAt[pos] = (uint8_t)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    for (uint32_t u = 0; u < tsize; u++) ct.st[cumul[symAt[u]]++] = (uint16_t)(tsize + u);
    uint32_t total = 0;
    for (uint32_t s = 0; s <= maxs; s++) {
        const int c = norm[s];
        if (c == 0) { ct.dnb[s] = ((tl + 1) << 16) - (1u << tl); ct.dfs[s] = 0; }
        else if (c == -1 || c == 1) { ct.dnb[s] = (tl << 16) - (1u << tl); ct.dfs[s] = (int32_t)total - 1; total++; }
        else {
            const uint32_t mbo = tl - hb32((uint32_t)c - 1);
            ct.dnb[s] = (mbo << 16) - ((uint32_t)c << mbo);
            ct.dfs[s] = (int32_t)total - c;
            total += (uint32_t)c;
        }
    }
}
__device__ __forceinline__ void fse_build_rle(LDSA Fse& ct, uint32_t sym) {
    ct.tlog = 0; ct.st[0] = 0; ct.dnb[sym] = 0; ct.dfs[sym] = 0;
}
__device__ __forceinline__ uint32_t fse_init_state(const LDSA Fse& ct, uint32_t sym) {
    const uint32_t nbo = (ct.dnb[sym] + (1u << 15)) >> 16;
    const uint32_t v = (nbo << 16) - ct.dnb[sym];
    return ct.st[(int32_t)(v >> nbo) + ct.dfs[sym]];
}
template <class Sink>
__device__ __forceinline__ void fse_encode(BitW<Sink>& b, const LDSA Fse& ct, uint32_t& state, uint32_t sym) {
    const uint32_t nbo = (state + ct.dnb[sym]) >> 16;
    b.add(state, nbo);
    state = ct.st[(int32_t)(state >> nbo) + ct.dfs[sym]];
}

// ---- Huffman (huf_compress.c), lane 0 only
// (RANK_POSITION_DISTINCT_COUNT_CUTOFF, huf_compress.c:455, is 158 + BIT_highbit32(158) = 165.  HUF_sort stores
// a symbol at region HUF_getIndex(count) + 1 (:577): its sort loop starts at region 165, the count-164 ties, and
// counts 165..255 are its region 166.  Buckets here are its regions minus one: bucket 165 holds counts 165..255
// and is sorted like the other log2 buckets)
__device__ __forceinline__ uint32_t huf_bucket(uint32_t c) { return c < 165 ? c : hb32(c) + 158; }
__device__ __forceinline__ HNode hget(const LDSA HNode* a) {
    HNode t;
    t.count = a->count; t.parent = a->parent; t.byte = a->byte; t.nb = a->nb;
    return t;
}
__device__ __forceinline__ void hset(LDSA HNode* a, const HNode& t) {
    a->count = t.count; a->parent = t.parent; a->byte = t.byte; a->nb = t.nb;
}
__device__ __forceinline__ void hswap(LDSA HNode* a, LDSA HNode* b) { const HNode t = hget(a); hset(a, hget(b)); hset(b, t); }
__device__ void huf_isort(LDSA HNode* a, int lo, int hi) {
    const int size = hi - lo + 1;
    a += lo;
    for (int i = 1; i < size; i++) {
        const HNode key = hget(&a[i]);
        int j = i - 1;
        while (j >= 0 && a[j].count < key.count) { hset(&a[j + 1], hget(&a[j])); j--; }
        hset(&a[j + 1], key);
    }
}
__device__ int huf_partition(LDSA HNode* a, int lo, int hi) {
    const uint32_t pivot = a[hi].count;
    int i = lo - 1;
    for (int jj = lo; jj < hi; jj++)
        if (a[jj].count > pivot) { i++; hswap(&a[i], &a[jj]); }
    hswap(&a[i + 1], &a[hi]);
    return i + 1;
}
// HUF_simpleQuickSort without recursion: a call task (lo, hi) insertion-sorts small ranges, else
// partitions in a loop that queues the smaller side as a call task and continues on the larger
// side; disjoint ranges sort independently, so the order tasks run in does not change the result
__device__ void huf_qsort(LDSA HNode* a, int lo0, int hi0, LDSA int32_t* stk) {
    int sp = 0;
    stk[sp++] = lo0;
    stk[sp++] = hi0;
    while (sp) {
        int hi = stk[--sp], lo = stk[--sp];
        if (hi - lo < 8) { huf_isort(a, lo, hi); continue; }
        while (lo < hi) {
            const int p = huf_partition(a, lo, hi);
            if (p - lo < hi - p) { stk[sp++] = lo; stk[sp++] = p - 1; lo = p + 1; }
            else { stk[sp++] = p + 1; stk[sp++] = hi; hi = p - 1; }
        }
    }
}
__device__ uint32_t huf_limit(LDSA HNode* node, uint32_t last, uint32_t maxNb, LDSA uint32_t* rankLast) {
    const uint32_t largest = node[last].nb;
    if (largest <= maxNb) return largest;
    int cost = 0;
    const uint32_t baseCost = 1u << (largest - maxNb);
    int n = (int)last;
    while (node[n].nb > maxNb) {
        cost += (int)(baseCost - (1u << (largest - node[n].nb)));
        node[n].nb = (uint8_t)maxNb;
        n--;
    }
    while (node[n].nb == maxNb) n--;
    cost >>= (largest - maxNb);
    const uint32_t NONE = 0xF0F0F0F0u;
    for (int i = 0; i < 14; i++) rankLast[i] = NONE;
    uint32_t curNb = maxNb;
    for (int p = n; p >= 0; p--) {
        if (node[p].nb >= curNb) continue;
        curNb = node[p].nb;
        rankLast[maxNb - curNb] = (uint32_t)p;
    }
    while (cost > 0) {
        uint32_t dec = hb32((uint32_t)cost) + 1;
        for (; dec > 1; dec--) {
            const uint32_t hi = rankLast[dec], lo = rankLast[dec - 1];
            if (hi == NONE) continue;
            if (lo == NONE) break;
            if (node[hi].count <= 2 * node[lo].count) break;
        }
        while (dec <= 12 && rankLast[dec] == NONE) dec++;
        cost -= 1 << (dec - 1);
        node[rankLast[dec]].nb++;
        if (rankLast[dec - 1] == NONE) rankLast[dec - 1] = rankLast[dec];
        if (rankLast[dec] == 0) rankLast[dec] = NONE;
        else {
            rankLast[dec]--;
            if (node[rankLast[dec]].nb != maxNb - dec) rankLast[dec] = NONE;
        }
    }
    while (cost < 0) {
        if (rankLast[1] == NONE) {
            while (node[n].nb == maxNb) n--;
            node[n + 1].nb--;
            rankLast[1] = (uint32_t)(n + 1);
            cost++;
            continue;
        }
        node[rankLast[1] + 1].nb--;
        rankLast[1]++;
        cost++;
    }
    return maxNb;
}
// HUF_buildCTable_wksp: fills L.nb / L.val, returns the table log
__device__ uint32_t huf_build(LDSA Lds& L, uint32_t maxs, uint32_t maxNb) {
    LDSA HNode* all = L.node;
    for (int i = 0; i < 514; i++) { all[i].count = 0; all[i].parent = 0; all[i].byte = 0; all[i].nb = 0; }
    LDSA HNode* node = all + 1;
    {   // HUF_sort: buckets, then quick sort of the log2 buckets
        // (bucket bounds in LDS, the sequence-code histograms' space: a private array indexed by
        // data would live in scratch memory)
        LDSA uint16_t* base = (LDSA uint16_t*)&L.cnt3[0][0];
        LDSA uint16_t* cur = base + 192;
        for (int b = 0; b < 192; b++) base[b] = 0;
        for (uint32_t s = 0; s <= maxs; s++) base[huf_bucket(L.cnt[s])]++;
        for (int b = 191; b > 0; b--) { base[b - 1] += base[b]; cur[b - 1] = base[b - 1]; }
        cur[191] = base[191];
        for (uint32_t s = 0; s <= maxs; s++) {
            const uint32_t r = huf_bucket(L.cnt[s]) + 1;
            const uint32_t p = cur[r]++;
            node[p].count = L.cnt[s];
            node[p].byte = (uint8_t)s;
        }
        for (uint32_t b = 165; b < 191; b++) {
            const uint32_t sz = (uint32_t)cur[b] - base[b];
            if (sz > 1) huf_qsort(node + base[b], 0, (int)sz - 1, L.qs);
        }
    }
    int nonNull = (int)maxs;
    while (node[nonNull].count == 0) nonNull--;
    int lowS = nonNull, nodeNb = 256;
    const int root = nodeNb + lowS - 1;
    int lowN = nodeNb;
    node[nodeNb].count = node[lowS].count + node[lowS - 1].count;
    node[lowS].parent = (uint16_t)nodeNb;
    node[lowS - 1].parent = (uint16_t)nodeNb;
    nodeNb++;
    lowS -= 2;
    for (int i = nodeNb; i <= root; i++) node[i].count = 1u << 30;
    all[0].count = 1u << 31;
    while (nodeNb <= root) {
        const int a = (node[lowS].count < node[lowN].count) ? lowS-- : lowN++;
        const int b = (node[lowS].count < node[lowN].count) ? lowS-- : lowN++;
        node[nodeNb].count = node[a].count + node[b].count;
        node[a].parent = (uint16_t)nodeNb;
        node[b].parent = (uint16_t)nodeNb;
        nodeNb++;
    }
    node[root].nb = 0;
    for (int i = root - 1; i >= 256; i--) node[i].nb = node[node[i].parent].nb + 1;
    for (int i = 0; i <= nonNull; i++) node[i].nb = node[node[i].parent].nb + 1;
    maxNb = huf_limit(node, (uint32_t)nonNull, maxNb, &L.cnt3[1][0]);
    LDSA uint16_t* nbPer = (LDSA uint16_t*)&L.cnt3[0][0];
    LDSA uint16_t* valPer = nbPer + 16;
    for (int i = 0; i < 13; i++) { nbPer[i] = 0; valPer[i] = 0; }
    for (int i = 0; i <= nonNull; i++) nbPer[node[i].nb]++;
    uint16_t mn = 0;
    for (int b = (int)maxNb; b > 0; b--) { valPer[b] = mn; mn += nbPer[b]; mn >>= 1; }
    for (int s = 0; s < 256; s++) { L.nb[s] = 0; L.val[s] = 0; }
    for (uint32_t i = 0; i <= maxs; i++) L.nb[node[i].byte] = node[i].nb;
    for (uint32_t s = 0; s <= maxs; s++) if (L.nb[s]) L.val[s] = valPer[L.nb[s]]++;
    return maxNb;
}
// HUF_compressWeights: FSE-compressed weights at o[pos..]; 0 = not compressible, 1 = rle
__device__ int huf_compress_weights(LDSA Lds& L, const LdsSink& o, int pos, uint32_t wn) {
    if (wn <= 1) return 0;
    LDSA uint32_t* cnt = L.cnt3[0];   // (free at this point)
    for (int s = 0; s < 13; s++) cnt[s] = 0;
    for (uint32_t i = 0; i < wn; i++) cnt[L.w[i]]++;
    uint32_t maxs = 12;
    while (!cnt[maxs]) maxs--;
    uint32_t big = 0;
    for (uint32_t s = 0; s <= maxs; s++) if (cnt[s] > big) big = cnt[s];
    if (big == wn) return 1;
    if (big == 1) return 0;
    const uint32_t tl = fse_opt_log(6, wn, maxs, 2);
    if (fse_normalize(L.norm, tl, cnt, wn, maxs, 0)) return 0;
    const int h = fse_write_ncount(o, pos, L.norm, maxs, tl);
    fse_build(L.fse[0], L.norm, maxs, tl, (LDSA uint8_t*)L.cnt3[1], L.cnt3[2]);
    if (wn <= 2) return 0;
    BitW<LdsSink> b{o, pos + h, 0, 0};
    uint32_t s1, s2;
    int i = (int)wn;
    if (wn & 1) {
        s1 = fse_init_state(L.fse[0], L.w[--i]);
        s2 = fse_init_state(L.fse[0], L.w[--i]);
        fse_encode(b, L.fse[0], s1, L.w[--i]);
    } else {
        s2 = fse_init_state(L.fse[0], L.w[--i]);
        s1 = fse_init_state(L.fse[0], L.w[--i]);
    }
    while (i > 0) {
        fse_encode(b, L.fse[0], s2, L.w[--i]);
        fse_encode(b, L.fse[0], s1, L.w[--i]);
    }
    b.add(s2, L.fse[0].tlog);
    b.add(s1, L.fse[0].tlog);
    return b.close() - pos;
}
// HUF_writeCTable_wksp into L.hdr; returns its size, -1 = not representable
__device__ int huf_write_table(LDSA Lds& L, uint32_t maxs, uint32_t tl) {
    for (uint32_t s = 0; s < maxs; s++) L.w[s] = L.nb[s] ? (uint8_t)(tl + 1 - L.nb[s]) : 0;
    const int h = huf_compress_weights(L, LdsSink{L.hdr}, 1, maxs);
    if (h > 1 && h < (int)(maxs / 2)) {
        L.hdr[0] = (uint8_t)h;
        return h + 1;
    }
    if (maxs > 128) return -1;
    L.hdr[0] = (uint8_t)(128 + maxs - 1);
    L.w[maxs] = 0;
    for (uint32_t s = 0; s < maxs; s += 2) L.hdr[s / 2 + 1] = (uint8_t)((L.w[s] << 4) + L.w[s + 1]);
    return (int)((maxs + 1) / 2 + 1);
}

// ---- wave helpers
// wave-wide scans through DPP row shifts + row broadcasts (no LDS round trip per step)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
    (void)lane;
    int x = (int)v;
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return (uint32_t)x;
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    return __builtin_amdgcn_readlane(wave_incl_scan(v, 0), 63);
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {   // (unsigned: 0 is the identity of a shifted-out lane)
    uint32_t x = v;
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false));
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false));
    return __builtin_amdgcn_readlane(x, 63);
}

// histogram of bytes [a, a+n) of src (4-aligned buffer) into cnt (256 bins), all lanes: 16 bytes
// per lane per round, bytes outside the range masked
__device__ void histo256(LDSA uint32_t* cnt, const Bytes& src, int a, int n, int lane) {
    for (int i = lane; i < 256; i += 64) cnt[i] = 0;
    wave_lds_fence();
    const int e = a + n;
    for (int base = a & ~3; base < e; base += 64 * 16) {
        const int p0 = base + 16 * lane;
        uint32_t w[4];   // (loads unconditional at clamped positions: one wait for the four)
#pragma unroll
        for (int d = 0; d < 4; d++) w[d] = ld_b32(src.r, (p0 + 4 * d < e ? p0 + 4 * d : (a & ~3)) + src.sh);
#pragma unroll
        for (int d = 0; d < 4; d++) {
            const int p = p0 + 4 * d;
            if (p < e) {
#pragma unroll
                for (int b = 0; b < 4; b++)
                    if (p + b >= a && p + b < e) atomicAdd((uint32_t*)&cnt[(w[d] >> (8 * b)) & 0xffu], 1u);
            }
        }
    }
    wave_lds_fence();
}
// (largest count, highest present symbol) of cnt[0..256)
__device__ void histo_stats(const LDSA uint32_t* cnt, int lane, uint32_t& largest, uint32_t& maxs) {
    uint32_t mx = 0, hi = 0;
    for (int i = 0; i < 4; i++) {
        const uint32_t c = cnt[lane * 4 + i];
        mx = max(mx, c);
        if (c) hi = (uint32_t)(lane * 4 + i) + 1;
    }
    largest = wave_max(mx);
    maxs = wave_max(hi);
    maxs = maxs ? maxs - 1 : 0;
}

// Huffman streams of lits[0, n) with the table (nb, val) into o[pos..]: 1 stream, or 4 with the
// jump table (HUF_compress1X/4X_usingCTable).  Each stream is assembled 64 symbols at a time:
// symbol i of a stream sits at bit (total - bits of symbols 0..i) -- the reference writes the last
// symbol first -- so a wave prefix sum places every code; codes are OR-ed into an LDS window
// of dwords and the window is stored to the aligned scratch `tmp`, then copied into place.
// Returns the streams' size, 0 = not possible (a stream over 64 KiB).
__device__ int huf_streams(LDSA Lds& L, const LDSA uint8_t* nb, const LDSA uint16_t* val, const Bytes& lits, int n,
                           int four, const Bytes& o, int pos, const Bytes& tmp, int lane) {
    const int nstreams = four ? 4 : 1;
    const int seg = four ? (n + 3) / 4 : n;
    int sizes[4] = {0, 0, 0, 0};
    uint32_t tbits[4] = {0, 0, 0, 0};
    // (4 symbols per lane: one unaligned dword of literals, bytes past the stream's end masked)
    for (int sidx = 0; sidx < nstreams; sidx++) {
        const int a = sidx * seg, e = (sidx == nstreams - 1) ? n : a + seg;
        uint32_t bits = 0;
        for (int i0 = a + 4 * lane; i0 < e; i0 += 1024) {   // (four dwords' loads in flight at once)
            uint32_t w[4];
#pragma unroll
            for (int u = 0; u < 4; u++) w[u] = lits.w32(i0 + 256 * u < e ? i0 + 256 * u : a);
#pragma unroll
            for (int u = 0; u < 4; u++)
#pragma unroll
                for (int k = 0; k < 4; k++) bits += i0 + 256 * u + k < e ? (uint32_t)nb[(w[u] >> (8 * k)) & 0xffu] : 0u;
        }
        bits = wave_sum(bits);
        tbits[sidx] = bits;
        sizes[sidx] = (int)((bits + 8) >> 3);
        if (four && sizes[sidx] > 65535) return 0;
    }
    {   // the caller rejects streams of n - 1 bytes or more (HUF_compressCTable_internal): skip them
        int tot = four ? 6 : 0;
        for (int sidx = 0; sidx < nstreams; sidx++) tot += sizes[sidx];
        if (tot >= n - 1) return 0;
    }
    int off = pos + (four ? 6 : 0);
    for (int sidx = 0; sidx < nstreams; sidx++) {
        const int a = sidx * seg, e = (sidx == nstreams - 1) ? n : a + seg;
        const uint32_t total = tbits[sidx];
        uint32_t carry = 0;            // bits of symbols before this group
        uint32_t cw = 0;               // pending partial dword (index cd), low part still open
        int cd = -1;
        uint32_t wn = lits.w32(a + 4 * lane < e ? a + 4 * lane : a);   // (the next group's dword, loaded a group ahead)
        for (int g = a; g < e; g += 256) {
            const int i = g + 4 * lane;
            const uint32_t w = wn;
            wn = lits.w32(i + 256 < e ? i + 256 : a);
            uint32_t len[4], code[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t sym = (w >> (8 * k)) & 0xffu;
                len[k] = i + k < e ? (uint32_t)nb[sym] : 0u;
                code[k] = val[sym];
            }
            const uint32_t L4 = len[0] + len[1] + len[2] + len[3];
            const uint32_t incl = wave_incl_scan(L4, lane);
            const uint32_t gsum = rdlane(incl, 63);
            const uint32_t hiBit = total - carry;              // group occupies [hiBit - gsum, hiBit)
            const uint32_t loBit = hiBit - gsum;
            const int d0 = (int)(loBit >> 5);
            const int d1 = (int)(((g == a ? hiBit + 1 : hiBit) + 31) >> 5);   // (+1: the end mark)
            for (int d = lane; d < d1 - d0; d += 64) L.stage[d] = 0;
            wave_lds_fence();
            // symbol i + k sits below the bits of every symbol before it in the group
            uint32_t S = incl - L4;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                S += len[k];
                if (len[k]) {
                    const uint32_t bp = hiBit - S - loBit + (loBit & 31u);   // bit offset in the window
                    const uint64_t v = (uint64_t)code[k] << (bp & 31u);
                    atomicOr((uint32_t*)&L.stage[bp >> 5], (uint32_t)v);
                    if ((uint32_t)(v >> 32)) atomicOr((uint32_t*)&L.stage[(bp >> 5) + 1], (uint32_t)(v >> 32));
                }
            }
            if (g == a && lane == 0) {
                const uint32_t bp = total - loBit + (loBit & 31u);
                atomicOr((uint32_t*)&L.stage[bp >> 5], 1u << (bp & 31u));
            }
            wave_lds_fence();
            if (cd >= 0 && lane == 0) atomicOr((uint32_t*)&L.stage[cd - d0], cw);
            wave_lds_fence();
            // store every window dword but the lowest unless the window ends on a dword boundary
            const bool last_group = g + 256 >= e;
            const int dstart = ((loBit & 31u) == 0 || last_group) ? d0 : d0 + 1;
            for (int d = dstart + lane; d < d1; d += 64) st_b32(tmp.r, 4 * d, L.stage[d - d0]);
            if (dstart != d0) { cw = L.stage[0]; cd = d0; } else { cd = -1; }
            carry += gsum;
            wave_lds_fence();
        }
        if (e == a) {   // empty stream: just the end mark
            if (lane == 0) st_b32(tmp.r, 0, 1u);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        copy_span(tmp, 0, o, off, sizes[sidx], lane, 64);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        off += sizes[sidx];
    }
    if (four && lane == 0) {
        for (int sidx = 0; sidx < 3; sidx++) { o.st8(pos + 2 * sidx, sizes[sidx] & 0xff); o.st8(pos + 2 * sidx + 1, sizes[sidx] >> 8); }
    }
    return off - pos;
}

}  // namespace ze

namespace ze {

// raw literals section (ZSTD_noCompressLiterals)
__device__ int lit_raw(const Bytes& att, const Bytes& lits, int n, int lane) {
    const int fl = 1 + (n > 31) + (n > 4095);
    if (lane == 0) {
        if (fl == 1) att.st8(0, (uint32_t)(n << 3) & 0xffu);
        else if (fl == 2) { const uint32_t v = (1u << 2) + ((uint32_t)n << 4); att.st8(0, v & 0xff); att.st8(1, v >> 8); }
        else { const uint32_t v = (3u << 2) + ((uint32_t)n << 4); att.st8(0, v & 0xff); att.st8(1, (v >> 8) & 0xff); att.st8(2, v >> 16); }
    }
    copy_span(lits, 0, att, fl, n, lane, 64);
    return n + fl;
}

// ZSTD_compressLiterals (zstd_compress_literals.c:70-159) with HUF_compress_internal
// (huf_compress.c:1177-1282) for the fast strategy; writes att[0..); returns the section size.
// newTable: the section uses a fresh table (left in L.nb / L.val)
__device__ int compress_literals(LDSA Lds& L, const Bytes& att, const Bytes& tmp, const Bytes& lits, int n, int ns,
                                 const zc::ZParams& P, int prevRepeat, int& newTable, int lane) {
    newTable = 0;
    ZEM_DECL;
    if (P.lit_off || n <= 63) return lit_raw(att, lits, n, lane);
    const int lh = 3 + (n >= 1024) + (n >= 16384);
    const int four = n >= 256;
    const int suspect = ns == 0 || n / ns >= 20;
    uint32_t largest, maxs;
    if (suspect && n >= 40960) {
        uint32_t b1, b2, m;
        histo256(L.cnt, lits, 0, 4096, lane);
        histo_stats(L.cnt, lane, b1, m);
        histo256(L.cnt, lits, n - 4096, 4096, lane);
        histo_stats(L.cnt, lane, b2, m);
        if (b1 + b2 <= ((2 * 4096) >> 7) + 4) return lit_raw(att, lits, n, lane);
    }
    histo256(L.cnt, lits, 0, n, lane);
    histo_stats(L.cnt, lane, largest, maxs);
    ZEM(0);   // literal histogram
    if (largest == (uint32_t)n) {                        // RLE literals
        const int fl = 1 + (n > 31) + (n > 4095);
        if (lane == 0) {
            if (fl == 1) att.st8(0, 1u + (((uint32_t)n << 3) & 0xffu));
            else if (fl == 2) { const uint32_t v = 1u + (1u << 2) + ((uint32_t)n << 4); att.st8(0, v & 0xff); att.st8(1, v >> 8); }
            else { const uint32_t v = 1u + (3u << 2) + ((uint32_t)n << 4); att.st8(0, v & 0xff); att.st8(1, (v >> 8) & 0xff); att.st8(2, v >> 16); }
            att.st8(fl, lits.b(0));
        }
        return fl + 1;
    }
    if (largest <= (uint32_t)(n >> 7) + 4) return lit_raw(att, lits, n, lane);
    int repeat = prevRepeat;
    if (repeat) {   // HUF_validateCTable
        bool bad = false;
        for (int i = 0; i < 4; i++) {
            const int s = lane * 4 + i;
            if (s <= (int)maxs && L.cnt[s] && !L.pnb[s]) bad = true;
        }
        if (ballot(bad)) repeat = 0;
    }
    const int minGain = (n >> 6) + 2;
    int c = 0, htype = 3;
    if (n <= 1024 && repeat) {
        c = huf_streams(L, L.pnb, L.pval, lits, n, four, att, lh, tmp, lane);
        if (c == 0 || c >= n - 1) return lit_raw(att, lits, n, lane);
    } else {
        if (lane == 0) {
            const uint32_t tl = huf_build(L, maxs, fse_opt_log(11, (uint32_t)n, maxs, 1));
            L.misc[0] = (uint32_t)huf_write_table(L, maxs, tl);
        }
        wave_lds_fence();
        const int h = (int)uni(L.misc[0]);
        ZEM(1);   // Huffman tree + table description
        if (h < 0) return lit_raw(att, lits, n, lane);
        bool useOld = false;
        if (repeat) {
            uint32_t o = 0, w = 0;
            for (int i = 0; i < 4; i++) {
                const int s = lane * 4 + i;
                if (s <= (int)maxs) { o += L.pnb[s] * L.cnt[s]; w += L.nb[s] * L.cnt[s]; }
            }
            const uint32_t oldS = wave_sum(o) >> 3, newS = wave_sum(w) >> 3;
            useOld = oldS <= (uint32_t)h + newS || h + 12 >= n;
        }
        if (useOld) {
            c = huf_streams(L, L.pnb, L.pval, lits, n, four, att, lh, tmp, lane);
            if (c == 0 || c >= n - 1) return lit_raw(att, lits, n, lane);
        } else {
            if (h + 12 >= n) return lit_raw(att, lits, n, lane);
            for (int i = lane; i < h; i += 64) att.st8(lh + i, L.hdr[i]);
            const int c2 = huf_streams(L, L.nb, L.val, lits, n, four, att, lh + h, tmp, lane);
            if (c2 == 0 || h + c2 >= n - 1) return lit_raw(att, lits, n, lane);
            c = h + c2;
            htype = 2;
        }
    }
    ZEM(2);   // Huffman streams
    if (c >= n - minGain) return lit_raw(att, lits, n, lane);
    newTable = htype == 2;
    if (lane == 0) {
        if (lh == 3) {
            const uint32_t v = (uint32_t)htype + ((uint32_t)four << 2) + ((uint32_t)n << 4) + ((uint32_t)c << 14);
            att.st8(0, v & 0xff); att.st8(1, (v >> 8) & 0xff); att.st8(2, v >> 16);
        } else if (lh == 4) {
            const uint32_t v = (uint32_t)htype + (2u << 2) + ((uint32_t)n << 4) + ((uint32_t)c << 18);
            att.st8(0, v & 0xff); att.st8(1, (v >> 8) & 0xff); att.st8(2, (v >> 16) & 0xff); att.st8(3, v >> 24);
        } else {
            const uint32_t v = (uint32_t)htype + (3u << 2) + ((uint32_t)n << 4) + ((uint32_t)c << 22);
            att.st8(0, v & 0xff); att.st8(1, (v >> 8) & 0xff); att.st8(2, (v >> 16) & 0xff); att.st8(3, v >> 24);
            att.st8(4, (uint32_t)c >> 10);
        }
    }
    return lh + c;
}

__device__ __forceinline__ void seq_unpack(uint32_t lo, uint32_t hi, uint32_t& ll, uint32_t& ml, uint32_t& off) {
    const uint64_t v = (uint64_t)lo | ((uint64_t)hi << 32);
    ll = (uint32_t)(v & 0xFFFFFu);
    ml = (uint32_t)((v >> 20) & 0xFFFFFu);
    off = (uint32_t)(v >> 40);
}

// sequences section after the nbSeq header (zstd_compress.c:2645-2689, ZSTD_buildSequencesStatistics,
// zstd_compress_sequences.c:157-382); att[pos..); returns its size, 0 = emit the block raw
__device__ int encode_sequences(LDSA Lds& L, const Bytes& att, const Bytes& tmp, int pos, rsrc_t seq, int ns, int lane) {
    ZEM_DECL;
    for (int i = lane; i < 3 * 64; i += 64) (&L.cnt3[0][0])[i] = 0;
    wave_lds_fence();
    for (int i = lane; i < ns; i += 64) {
        uint32_t ll, ml, off;
        seq_unpack(ld_b32(seq, 8 * i), ld_b32(seq, 8 * i + 4), ll, ml, off);
        atomicAdd((uint32_t*)&L.cnt3[0][ll_code(ll)], 1u);
        atomicAdd((uint32_t*)&L.cnt3[1][hb32(off)], 1u);
        atomicAdd((uint32_t*)&L.cnt3[2][ml_code(ml - 3)], 1u);
    }
    wave_lds_fence();
    ZEM(3);   // sequence histograms
    // codes of the first and the last sequence (RLE tables, FSE count trick)
    uint32_t c0[3], cl[3];
    {
        uint32_t ll, ml, off;
        seq_unpack(ld_b32(seq, 0), ld_b32(seq, 4), ll, ml, off);
        c0[0] = ll_code(ll); c0[1] = hb32(off); c0[2] = ml_code(ml - 3);
        seq_unpack(ld_b32(seq, 8 * (ns - 1)), ld_b32(seq, 8 * (ns - 1) + 4), ll, ml, off);
        cl[0] = ll_code(ll); cl[1] = hb32(off); cl[2] = ml_code(ml - 3);
    }
    int op = pos;
    if (lane == 0) {
        const uint32_t maxTab[3] = {35, 31, 52}, fseLog[3] = {9, 8, 9}, defLog[3] = {6, 5, 6}, defMax[3] = {35, 28, 52};
        const int head = op++;
        uint32_t types[3];
        int lastCount = 0;
        for (int t = 0; t < 3; t++) {
            LDSA uint32_t* cnt = L.cnt3[t];
            uint32_t maxs = maxTab[t];
            while (!cnt[maxs]) maxs--;
            uint32_t big = 0;
            for (uint32_t s = 0; s <= maxs; s++) big = max(big, cnt[s]);
            const int defOk = t == 1 ? (maxs <= 28) : 1;
            int ty;   // ZSTD_selectEncodingType, strategy < ZSTD_lazy
            if (big == (uint32_t)ns) ty = (defOk && ns <= 2) ? 0 : 1;
            else {
                ty = 2;
                if (defOk) {
                    const uint32_t dynMin = ((1u << defLog[t]) * 9) >> 3;
                    if ((uint32_t)ns < dynMin || big < ((uint32_t)ns >> (defLog[t] - 1))) ty = 0;
                }
            }
            types[t] = (uint32_t)ty;
            if (ty == 1) {
                fse_build_rle(L.fse[t], maxs);
                att.st8(op++, c0[t]);
            } else if (ty == 0) {
                for (uint32_t s = 0; s <= defMax[t]; s++) L.norm[s] = t == 0 ? kLLDef[s] : (t == 1 ? kOFDef[s] : kMLDef[s]);
                fse_build(L.fse[t], L.norm, defMax[t], defLog[t], L.symAt, L.cumul);
            } else {
                uint32_t n1 = (uint32_t)ns;
                const uint32_t tl = fse_opt_log(fseLog[t], (uint32_t)ns, maxs, 2);
                if (cnt[cl[t]] > 1) { cnt[cl[t]]--; n1--; }
                fse_normalize(L.norm, tl, cnt, n1, maxs, n1 >= 2048);
                const int h = fse_write_ncount(att, op, L.norm, maxs, tl);
                fse_build(L.fse[t], L.norm, maxs, tl, L.symAt, L.cumul);
                op += h;
                lastCount = h;
            }
        }
        att.st8(head, (types[0] << 6) + (types[1] << 4) + (types[2] << 2));
        L.misc[1] = (uint32_t)op;
        L.misc[2] = (uint32_t)lastCount;
    }
    wave_lds_fence();
    op = (int)uni(L.misc[1]);
    const int lastCount = (int)uni(L.misc[2]);
    // ZSTD_encodeSequences_body (zstd_compress_sequences.c:268-382), the last sequence first, 64
    // sequences at a time.  The three FSE state chains (offset, match length, literal length) are
    // independent: lanes 0 / 1 / 2 run one each (one dependent LDS lookup per sequence), leaving every
    // sequence's (nbBits, bits) per table in LDS; then every lane places its sequence's six fields --
    // OF / ML / LL state bits, LL / ML / OF extra bits, in the reference's order -- at bit offsets from
    // a wave suffix sum, OR-ed into an LDS window of dwords that leaves for the aligned scratch `tmp`.
    // The stream is copied behind the table descriptions at the end.
    ZEM(4);   // FSE tables
    const int tb = lane == 0 ? 1 : (lane == 1 ? 2 : 0);     // chain lane -> table (OF, ML, LL)
    uint32_t state = 0;
    uint32_t bitpos = 0;          // stream bits written so far
    uint32_t cw = 0;              // the open (partial) dword at bitpos >> 5
    uint32_t q0, q1;              // the group's sequence, loaded a group ahead
    {
        const int x = min(max(ns - 64, 0) + lane, ns - 1);
        q0 = ld_b32(seq, 8 * x); q1 = ld_b32(seq, 8 * x + 4);
    }
    for (int g = ns; g > 0; g -= 64) {
        const int g0 = g >= 64 ? g - 64 : 0, gn = g - g0;
        const int i = lane;
        uint32_t ll = 0, ml = 3, off = 0;
        if (i < gn) seq_unpack(q0, q1, ll, ml, off);
        {
            const int x = min((g0 >= 64 ? g0 - 64 : 0) + lane, max(g0 - 1, 0));
            q0 = ld_b32(seq, 8 * x); q1 = ld_b32(seq, 8 * x + 4);
        }
        const uint32_t llc = ll_code(ll), ofc = hb32(max(off, 1u)), mlc = ml_code(ml - 3);
        // per table and sequence (deltaNbBits, deltaFindState) into LDS (the Huffman sort stack, free
        // by now): the chain lanes read them ahead of the state-dependent lookups
        {
            LDSA uint32_t* cd = (LDSA uint32_t*)L.qs;
            cd[2 * i] = L.fse[1].dnb[ofc];             cd[2 * i + 1] = (uint32_t)L.fse[1].dfs[ofc];
            cd[128 + 2 * i] = L.fse[2].dnb[mlc];       cd[128 + 2 * i + 1] = (uint32_t)L.fse[2].dfs[mlc];
            cd[256 + 2 * i] = L.fse[0].dnb[llc];       cd[256 + 2 * i + 1] = (uint32_t)L.fse[0].dfs[llc];
        }
        wave_lds_fence();
        // ---- state chains (lanes 0..2: OF, ML, LL; the other lanes repeat lane 2's), sequences gn-1 .. 0
        {
            const LDSA uint16_t* st = L.fse[tb].st;
            const LDSA uint32_t* cdt = (const LDSA uint32_t*)L.qs + 128 * (lane < 3 ? lane : 2);
            int k = gn - 1;
            if (g0 + k == ns - 1) {                           // FSE_initCState2 (no bits)
                const uint32_t dn = cdt[2 * k];
                const int32_t df = (int32_t)cdt[2 * k + 1];
                const uint32_t nbo = (dn + (1u << 15)) >> 16;
                const uint32_t v = (nbo << 16) - dn;
                state = st[(int32_t)(v >> nbo) + df];
                if (lane < 3) L.sq[3 * k + lane] = 0u;
                k--;
            }
            auto step = [&](uint32_t dn, int32_t df, int kk) {   // FSE_encodeSymbol
                const uint32_t nbo = (state + dn) >> 16;
                const uint32_t outw = (nbo << 16) | (state & ((1u << nbo) - 1u));
                state = st[(int32_t)(state >> nbo) + df];
                if (lane < 3) L.sq[3 * kk + lane] = outw;
            };
            for (; k >= 3; k -= 4) {                          // (the table deltas of 4 steps read up front)
                const uint32_t d0 = cdt[2 * k], f0 = cdt[2 * k + 1], d1 = cdt[2 * k - 2], f1 = cdt[2 * k - 1],
                               d2 = cdt[2 * k - 4], f2 = cdt[2 * k - 3], d3 = cdt[2 * k - 6], f3 = cdt[2 * k - 5];
                step(d0, (int32_t)f0, k);
                step(d1, (int32_t)f1, k - 1);
                step(d2, (int32_t)f2, k - 2);
                step(d3, (int32_t)f3, k - 3);
            }
            for (; k >= 0; k--) step(cdt[2 * k], (int32_t)cdt[2 * k + 1], k);
        }
        wave_lds_fence();
        ZEM(5);   // state chains
        // ---- fields of sequence i, its bit offset (the group is written from its last sequence down)
        const uint32_t wOF = i < gn ? L.sq[3 * i] : 0u, wML = i < gn ? L.sq[3 * i + 1] : 0u, wLL = i < gn ? L.sq[3 * i + 2] : 0u;
        const uint32_t nOF = wOF >> 16, nML = wML >> 16, nLL = wLL >> 16;
        const uint32_t nll = i < gn ? ll_bits(ll) : 0u, nml = i < gn ? ml_bits(ml - 3) : 0u, nof = i < gn ? ofc : 0u;
        const uint32_t T = nOF + nML + nLL + nll + nml + nof;
        const uint32_t incl = wave_incl_scan(T, lane);
        const uint32_t gbits = rdlane(incl, 63);
        const uint32_t base = bitpos & ~31u;
        uint32_t p = bitpos + (gbits - incl) - base;          // window-relative start of sequence i
        const int nd = (int)((bitpos - base + gbits + 31) >> 5) + 1;
        for (int d = lane; d < nd; d += 64) L.stage[d] = d == 0 ? cw : 0u;
        wave_lds_fence();
        auto put = [&](uint32_t v, uint32_t n) {
            if (n) {
                v &= n >= 32 ? ~0u : ((1u << n) - 1u);
                const uint64_t x = (uint64_t)v << (p & 31u);
                atomicOr((uint32_t*)&L.stage[p >> 5], (uint32_t)x);
                if ((uint32_t)(x >> 32)) atomicOr((uint32_t*)&L.stage[(p >> 5) + 1], (uint32_t)(x >> 32));
            }
            p += n;
        };
        put(wOF & 0xffffu, nOF);
        put(wML & 0xffffu, nML);
        put(wLL & 0xffffu, nLL);
        put(ll, nll);
        put(ml - 3, nml);
        put(off, nof);
        wave_lds_fence();
        const uint32_t end = bitpos + gbits;
        const int full = (int)((end - base) >> 5);            // complete dwords of the window
        for (int d = lane; d < full; d += 64) st_b32(tmp.r, (int)(base >> 3) + 4 * d, L.stage[d]);
        cw = L.stage[full];
        bitpos = end;
        wave_lds_fence();
        ZEM(6);   // field packing
    }
    // FSE_flushCState x 3 (ML, OF, LL), BIT_closeCStream (the end mark), into the open dword
    int res = 0;
    {
        const uint32_t sML = (uint32_t)__builtin_amdgcn_readlane((int)state, 1), sOF = (uint32_t)__builtin_amdgcn_readlane((int)state, 0),
                       sLL = (uint32_t)__builtin_amdgcn_readlane((int)state, 2);
        uint64_t acc = cw;
        uint32_t nb = bitpos & 31u;
        const uint32_t base = bitpos & ~31u;
        const uint32_t tl2 = L.fse[2].tlog, tl1 = L.fse[1].tlog, tl0 = L.fse[0].tlog;
        // (at most 31 + 3 x 9 + 1 = 59 bits: one u64)
        acc |= (uint64_t)(sML & ((1u << tl2) - 1u)) << nb; nb += tl2;
        acc |= (uint64_t)(sOF & ((1u << tl1) - 1u)) << nb; nb += tl1;
        acc |= (uint64_t)(sLL & ((1u << tl0) - 1u)) << nb; nb += tl0;
        acc |= 1ull << nb; nb += 1;
        if (lane == 0) {
            st_b32(tmp.r, (int)(base >> 3), (uint32_t)acc);
            if (nb > 32) st_b32(tmp.r, (int)(base >> 3) + 4, (uint32_t)(acc >> 32));
        }
        const int bs = (int)((base + nb + 7) >> 3);          // stream bytes
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        copy_span(tmp, 0, att, op, bs, lane, 64);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        res = (lastCount && lastCount + bs < 4) ? 0 : op + bs - pos;
    }
    return res;
}

}  // namespace ze

// one wave per frame; block k of every frame: entropy coding, block decision, frame assembly
extern "C" __global__ void __launch_bounds__(64)
lzh_zstd_entropy_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size, int level, int k,
                        uint8_t* scratch, uint64_t fstride, uint64_t seq_off, uint64_t lit_off, uint64_t att_off,
                        uint64_t tmp_off, uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t f0) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_raw[(sizeof(ze::Lds) + 3) / 4];
    LDSA ze::Lds& L = *(LDSA ze::Lds*)lds_raw;
    const int lane = threadIdx.x;
    const uint64_t f = (uint64_t)blockIdx.x + f0;
    const uint64_t ioff = f * chunk_size;
    if (ioff >= n_total && !(n_total == 0 && f == 0)) return;
    const uint64_t nf = n_total ? min(chunk_size, n_total - ioff) : 0;
    const ZParams P = params_for(level, nf);
    if (!P.ok) return;
    const uint64_t nblocks = nf ? (nf + P.bsize - 1) / P.bsize : 1;
    if ((uint64_t)k >= nblocks) return;
    uint8_t* fs = scratch + f * fstride;
    rsrc_t hdr = make_rsrc(fs, 1024);
    Bytes out;
    out.init(stage + f * stride, stride);
    int out_off;
    if (k == 0) {
        // ZSTD_writeFrameHeader (zstd_compress.c:4012-4058): single segment, content size, no checksum
        const uint64_t wsize = 1ull << P.wlog;
        const int single = wsize >= nf;
        const int fcs = (nf >= 256) + (nf >= 65536 + 256) + (nf >= 0xFFFFFFFFull);
        int o = 0;
        if (lane == 0) {
            out.st8(0, 0x28); out.st8(1, 0xB5); out.st8(2, 0x2F); out.st8(3, 0xFD);
            out.st8(4, (uint32_t)((single << 5) + (fcs << 6)));
        }
        o = 5;
        if (!single) { if (lane == 0) out.st8(o, (P.wlog - 10) << 3); o++; }
        if (lane == 0) {
            if (fcs == 0) { if (single) out.st8(o, (uint32_t)nf & 0xff); }
            else if (fcs == 1) { const uint32_t v = (uint32_t)(nf - 256); out.st8(o, v & 0xff); out.st8(o + 1, v >> 8); }
            else if (fcs == 2) { for (int i = 0; i < 4; i++) out.st8(o + i, (uint32_t)(nf >> (8 * i)) & 0xff); }
            else { for (int i = 0; i < 8; i++) out.st8(o + i, (uint32_t)(nf >> (8 * i)) & 0xff); }
        }
        o += fcs == 0 ? (single ? 1 : 0) : (fcs == 1 ? 2 : (fcs == 2 ? 4 : 8));
        out_off = o;
        if (lane == 0) { st_b32(hdr, 16, 1u); st_b32(hdr, 20, 4u); st_b32(hdr, 24, 0u); }
    } else {
        out_off = (int)uni(ld_b32(hdr, 28));
    }
    if (nf == 0) {                                        // ZSTD_writeEpilogue: empty last raw block
        if (lane == 0) { out.st8(out_off, 1); out.st8(out_off + 1, 0); out.st8(out_off + 2, 0); csizes[f] = (uint32_t)out_off + 3; }
        return;
    }
    const int bs = k * (int)P.bsize;
    const int be = (int)min<uint64_t>(nf, (uint64_t)bs + P.bsize);
    const int len = be - bs;
    const int last = (uint64_t)be == nf;
    Bytes in_b;
    in_b.init(in + ioff, min<uint64_t>(in_readable - ioff, nf + 16));
    const int skip = len < 7 || uni(ld_b32(hdr, 32)) != 0u;
    int csize = 0, newTable = 0;
    Bytes att;
    att.init(fs + att_off, tmp_off - att_off);
    if (!skip) {
        const int ns = (int)uni(ld_b32(hdr, 0)), nl = (int)uni(ld_b32(hdr, 4));
        const int prevRepeat = (int)uni(ld_b32(hdr, 24));
        if (prevRepeat) {
            rsrc_t ht = make_rsrc(fs + zc::kHufOff, 768);
            for (int s = lane; s < 256; s += 64) {
                L.pnb[s] = (uint8_t)ld_u8(ht, s);
                L.pval[s] = (uint16_t)(ld_u8(ht, 256 + 2 * s) | (ld_u8(ht, 257 + 2 * s) << 8));
            }
            wave_lds_fence();
        }
        Bytes lits, tmp;
        lits.init(fs + lit_off, P.bsize + 64);
        tmp.init(fs + tmp_off, P.bsize + 256);
        int o = ze::compress_literals(L, att, tmp, lits, nl, ns, P, prevRepeat, newTable, lane);
        if (lane == 0) {
            if (ns < 128) att.st8(o, (uint32_t)ns);
            else if (ns < 0x7F00) { att.st8(o, (uint32_t)((ns >> 8) + 0x80)); att.st8(o + 1, (uint32_t)ns & 0xff); }
            else { att.st8(o, 0xFF); att.st8(o + 1, (uint32_t)(ns - 0x7F00) & 0xff); att.st8(o + 2, (uint32_t)(ns - 0x7F00) >> 8); }
        }
        o += ns < 128 ? 1 : (ns < 0x7F00 ? 2 : 3);
        if (ns) {
            const int sz = ze::encode_sequences(L, att, tmp, o, make_rsrc(fs + seq_off, (uint32_t)(lit_off - seq_off)), ns, lane);
            csize = sz ? o + sz : 0;
        } else {
            csize = o;
        }
        if (csize && csize >= len - ((len >> 6) + 2)) csize = 0;   // ZSTD_minGain
    }
    if (len >= 7 && k > 0 && csize < 25) {                          // RLE block (not for the first block)
        const uint32_t b0 = in_b.b(bs);
        bool diff = false;
        for (int i = lane; i < len; i += 64) diff |= in_b.b(bs + i) != b0;
        if (!ballot(diff)) csize = 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int bsz;
    if (csize == 0) {
        if (lane == 0) { const uint32_t h = (uint32_t)last + ((uint32_t)len << 3); out.st8(out_off, h & 0xff); out.st8(out_off + 1, (h >> 8) & 0xff); out.st8(out_off + 2, h >> 16); }
        copy_span(in_b, bs, out, out_off + 3, len, lane, 64);
        bsz = 3 + len;
    } else if (csize == 1) {
        if (lane == 0) {
            const uint32_t h = (uint32_t)last + (1u << 1) + ((uint32_t)len << 3);
            out.st8(out_off, h & 0xff); out.st8(out_off + 1, (h >> 8) & 0xff); out.st8(out_off + 2, h >> 16);
            out.st8(out_off + 3, in_b.b(bs));
        }
        bsz = 4;
    } else {
        if (lane == 0) { const uint32_t h = (uint32_t)last + (2u << 1) + ((uint32_t)csize << 3); out.st8(out_off, h & 0xff); out.st8(out_off + 1, (h >> 8) & 0xff); out.st8(out_off + 2, h >> 16); }
        copy_span(att, 0, out, out_off + 3, csize, lane, 64);
        bsz = 3 + csize;
        // confirm repcodes and the Huffman table (ZSTD_blockState_confirmRepcodesAndEntropyTables)
        if (lane == 0) { st_b32(hdr, 16, ld_b32(hdr, 8)); st_b32(hdr, 20, ld_b32(hdr, 12)); }
        if (newTable) {
            rsrc_t ht = make_rsrc(fs + zc::kHufOff, 768);
            for (int s = lane; s < 256; s += 64) {
                st_u8(ht, s, L.nb[s]);
                st_u8(ht, 256 + 2 * s, L.val[s] & 0xff);
                st_u8(ht, 257 + 2 * s, L.val[s] >> 8);
            }
            if (lane == 0) st_b32(hdr, 24, 1u);
        }
    }
    out_off += bsz;
    if (lane == 0) {
        st_b32(hdr, 28, (uint32_t)out_off);
        if (last) csizes[f] = (uint32_t)out_off;
    }
}

#include "launch.h"
#include <algorithm>

#if LZH_ZSTDC_STATS
extern "C" int lzh_debug_zstdc_stats(unsigned long long* host, int reset) {
    if (reset) {
        unsigned long long z[24] = {};
        return hipMemcpyToSymbol(HIP_SYMBOL(zc::lzh_zstdc_stats_buf), z, sizeof(z)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(zc::lzh_zstdc_stats_buf), 24 * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#endif

size_t lzh_zstd_scratch_stride(size_t chunk_size, int level) {
    const ZParams P = params_for(level, chunk_size);
    if (!P.ok) return 0;
    // the tail chunk may use a larger table (smaller chunks select other clevels rows)
    uint32_t hmax = P.hlog;
    for (int lg = 6; lg <= 31 && (1ull << (lg - 1)) < chunk_size; lg++) {
        const ZParams Q = params_for(level, std::min<uint64_t>(chunk_size, 1ull << lg));
        if (Q.ok) hmax = std::max(hmax, Q.hlog);
    }
    const ZParams T = params_for(level, 1);
    if (T.ok) hmax = std::max(hmax, T.hlog);
    return (size_t)layout_for(P.bsize, hmax).stride;
}

int lzh_zstd_level_ok(int level, size_t chunk_size) {
    // every chunk size up to chunk_size must map to a fast-strategy row
    for (uint64_t n : {(uint64_t)chunk_size, (uint64_t)16384, (uint64_t)131072, (uint64_t)262144, (uint64_t)1})
        if (n <= chunk_size && !params_for(level, n).ok) return 0;
    return 1;
}

// the split of single-block frames over the side stream (0: every launch on the caller's stream)
static int g_zstdc_split = 1;
extern "C" int lzh_debug_zstdc_split(int on) {
    g_zstdc_split = on ? 1 : 0;
    return 0;
}

hipError_t lzh_launch_zstd_compress(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                    int level, uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks,
                                    uint8_t* scratch, hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    const ZParams P = params_for(level, std::min<uint64_t>(chunk_size, n_total ? n_total : 0));
    if (!P.ok) return hipErrorInvalidValue;
    const ZParams PF = params_for(level, chunk_size);
    const size_t fstride = lzh_zstd_scratch_stride(chunk_size, level);
    const Layout Lo = layout_for(PF.bsize, 16);   // offsets below tab_off do not depend on hlog
    const uint32_t nblocks = (uint32_t)((std::min<uint64_t>(chunk_size, std::max<uint64_t>(n_total, 1)) + PF.bsize - 1) / PF.bsize);
#ifndef LZH_ZSTD_LDS_MAX
#define LZH_ZSTD_LDS_MAX 65536u   // largest hash table kept in LDS (else in the frame's scratch, via L2)
#endif
    // 3-byte entries (LdsTab24) below 16 MiB chunks, else 4-byte ones
    // (17-bit entries, LdsTab17, for chunks of at most 128 KiB)
    const uint32_t ebytes = chunk_size < (16u << 20) ? 3u : 4u;
    const uint32_t t17 = (2u << PF.hlog) + std::max((1u << PF.hlog) / 8u, 4u);
    const uint32_t lds_tab = (4u << PF.hlog) > (uint32_t)LZH_ZSTD_LDS_MAX ? 0u
                             : (LZH_ZSTD_TAB17 && chunk_size <= 131072u) ? ((t17 + 15u) & ~15u) : (ebytes << PF.hlog);
    auto match = [&](hipStream_t st, uint32_t k, uint32_t f0, uint32_t nf) {
        hipLaunchKernelGGL(lzh_zstd_match_kernel, dim3(nf), dim3(64), lds_tab, st, in, n_total, in_readable,
                           chunk_size, level, (int)k, scratch, (uint64_t)fstride, Lo.seq_off, Lo.lit_off, Lo.tab_off,
                           lds_tab, f0);
    };
    auto entropy = [&](hipStream_t st, uint32_t k, uint32_t f0, uint32_t nf) {
        hipLaunchKernelGGL(lzh_zstd_entropy_kernel, dim3(nf), dim3(64), 0, st, in, n_total, in_readable,
                           chunk_size, level, (int)k, scratch, (uint64_t)fstride, Lo.seq_off, Lo.lit_off, Lo.att_off,
                           Lo.tmp_off, stage, stride, csizes, f0);
    };
    // Single-block frames: a frame's entropy stage needs only its own match stage, so the frames split in
    // two.  The first half runs match + entropy on the caller stream's high-priority side stream (its waves go
    // out first), the second half's match on the caller's stream beside it; the first half's entropy then
    // runs beside the second half's matching and only the second half's entropy is left at the end.
    hipStream_t sq = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    if (g_zstdc_split && std::max(nblocks, 1u) == 1 && nchunks >= 2 && lzh_side_stream(s, sq, fork, join)) {
        const uint32_t h = nchunks / 2;
        (void)hipEventRecord(fork, s);
        (void)hipStreamWaitEvent(sq, fork, 0);
        match(sq, 0, 0, h);
        match(s, 0, h, nchunks - h);
        entropy(sq, 0, 0, h);
        (void)hipEventRecord(join, sq);
        entropy(s, 0, h, nchunks - h);
        (void)hipStreamWaitEvent(s, join, 0);
        return hipGetLastError();
    }
    for (uint32_t k = 0; k < std::max(nblocks, 1u); k++) {
        match(s, k, 0, nchunks);
        entropy(s, k, 0, nchunks);
    }
    return hipGetLastError();
}
