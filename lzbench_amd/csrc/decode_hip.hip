// lzbench_amd/csrc/decode_hip.hip -- LZ4 and snappy block decoders for gfx950.
//
// One 64-lane wavefront per chunk.  The compressed stream is read from a 512-byte register
// window (two VGPRs across the wave: v_readlane / ds_bpermute, no memory round trip); the
// last 4 KiB of decoded output stay in an LDS window (match sources there are LDS-to-LDS
// copies) and leave for HBM as aligned dword stores; far match sources are read back from the
// already-flushed output with L1-bypassing loads.  Sequences / tags are decoded a group at a
// time (groups::), with a checked one-at-a-time path for everything a group does not take.
//
// Acceptance rules follow the reference decoders so malformed input is rejected:
//   LZ4_decompress_safe   /root/reference/lz4/lz4.c:1707-1729, :1929-2151, :2170-2176
//   snappy RawUncompress  /root/reference/snappy/snappy.cc:819-1036, :1319-1407
// (lzbench itself calls LZ4_decompress_fast, compressors.cpp:358-362, which trusts its
// input; on valid streams both produce identical bytes.)
#include "common.h"

// Debug counters (-DLZH_DEC_STATS=1 builds only, read by tools/dec_stats.py): per-wave sums in LDS,
// added to a device array when the chunk ends.
#ifndef LZH_DEC_STATS
#define LZH_DEC_STATS 0
#endif
#if LZH_DEC_STATS
__shared__ unsigned long long g_dst[16];
__device__ unsigned long long lzh_dec_stats_buf[16];
#define DST(i, v) do { if (threadIdx.x == 0) g_dst[i] += (unsigned long long)(v); } while (0)
#define DCLK(t) const uint64_t t = __builtin_amdgcn_s_memtime()
#else
#define DST(i, v) do {} while (0)
#define DCLK(t) do {} while (0)
#endif
#ifdef LZH_ISA_MARKS
#define DMARK(i) asm volatile("; DMARK " #i ::: "memory")
#else
#define DMARK(i) ((void)0)
#endif

namespace {

#ifndef LZH_DEC_RING
#define LZH_DEC_RING 1
#endif
constexpr int kRingBytes = 512 + 16;   // LDS copy of a window: ring over offsets mod 512 + mirror

// Register window over a byte stream (512 bytes in two VGPRs across the wave) with an LDS copy
// (ring indexed by descriptor offset mod 512, its first 16 bytes mirrored past the end): uniform
// reads use v_readlane on the registers, per-lane reads one LDS load instead of cross-lane
// permutes of both registers.
template <bool kRing>
struct WinT {
    rsrc_t r;
    int sh;       // descriptor offset of stream byte 0
    int wb;       // descriptor offset (4-aligned) of the window start
    uint32_t w0, w1;
    LDSA uint8_t* ring;
    __device__ __forceinline__ void bind(const Bytes& b, LDSA uint8_t* rg) { r = b.r; sh = b.sh; ring = rg; }
    __device__ __forceinline__ void put_ring(int D, uint32_t v) const {
        if (!(LZH_DEC_RING && kRing)) return;
        const int i = D & 511;
        *(volatile LDSA uint32_t*)(ring + i) = v;
        if (i < 16) *(volatile LDSA uint32_t*)(ring + 512 + i) = v;
    }
    __device__ __forceinline__ void load(int pos, int lane) {
        wb = (pos + sh) & ~3;
        w0 = ld_b32(r, wb + 4 * lane);
        w1 = ld_b32(r, wb + 256 + 4 * lane);
        put_ring(wb + 4 * lane, w0);
        put_ring(wb + 256 + 4 * lane, w1);
    }
    // make stream bytes [pos, pos+16) addressable
    __device__ __forceinline__ void ensure(int pos, int lane) {
        const int x = pos + sh;
        if (x >= wb && x + 16 <= wb + 512) return;
        if (x >= wb + 256 && x + 16 <= wb + 768) {
            w0 = w1;
            wb += 256;
            w1 = ld_b32(r, wb + 256 + 4 * lane);
            put_ring(wb + 256 + 4 * lane, w1);
            return;
        }
        load(pos, lane);
    }
    __device__ __forceinline__ uint32_t byte(int pos) const {
        const int x = pos + sh;
        const int d = (x - wb) >> 2;
        const uint32_t v = d < 64 ? rdlane(w0, d) : rdlane(w1, d - 64);
        return (v >> (8 * (x & 3))) & 0xffu;
    }
    __device__ __forceinline__ bool covers(int p0, int p1) const { return p0 + sh >= wb && p1 + sh <= wb + 512; }
    // per-lane 4 bytes at stream position pos (pos .. pos+3 inside the window)
    __device__ __forceinline__ uint32_t lane_word(int pos) const {
        const int x = pos + sh;
        if (LZH_DEC_RING && kRing) {
            const int a = x & 508;
            const uint32_t lo = *(volatile const LDSA uint32_t*)(ring + a), hi = *(volatile const LDSA uint32_t*)(ring + a + 4);
            return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)x & 3u);
        }
        const int d = (x - wb) >> 2;
        const uint32_t a0 = lane_gather(w0, d & 63), a1 = lane_gather(w1, d & 63);
        const uint32_t b0 = lane_gather(w0, (d + 1) & 63), b1 = lane_gather(w1, (d + 1) & 63);
        const uint32_t lo = d < 64 ? a0 : a1, hi = d + 1 < 64 ? b0 : b1;
        return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)x & 3u);
    }
    // per-lane byte at stream position pos (inside the window) via cross-lane permute
    __device__ __forceinline__ uint32_t lane_byte(int pos) const {
        const int x = pos + sh;
        if (LZH_DEC_RING && kRing) return ((volatile const LDSA uint8_t*)ring)[x & 511];
        const int d = (x - wb) >> 2;
        const uint32_t a = lane_gather(w0, d & 63), b = lane_gather(w1, d & 63);
        return ((d < 64 ? a : b) >> (8 * (x & 3))) & 0xffu;
    }
};

typedef WinT<true> Win;     // lz4 / snappy decoders
typedef WinT<false> ZWin;   // zstd (its LDS budget has no room for rings: 8 waves per CU)

__device__ __forceinline__ void copy_raw(const Bytes& in, const Bytes& out, int len, int lane) {
    copy_span(in, 0, out, 0, len, lane, LZH_WAVE);
}

}  // namespace

// ---------------------------------------------------------------------------------------
// Output through an LDS window.  The last kW decoded bytes of the chunk stay in LDS, so a
// match whose source lies in them is an LDS-to-LDS copy with no memory round trip; decoded
// bytes leave for global memory as aligned dword stores once 256 are pending.  Far matches read
// the (already flushed) output with L1-bypassing loads.
namespace owin {

#ifndef LZH_DEC_KW
#define LZH_DEC_KW 4096
#endif
#ifndef LZH_DEC_WIDE
#define LZH_DEC_WIDE 2   // wider output windows for launches with few chunks: 0 off, 1 up to 8 KiB, 2 up to 16 KiB
#endif
constexpr int kW = LZH_DEC_KW;   // LDS output window bytes (power of two)

template <int KW>
struct SinkT {
    static constexpr int kWin = KW;
    LDSA uint8_t* b;
    Bytes out;
    int flushed;      // output bytes [0, flushed) are in global memory
    int ringlo;       // output bytes [ringlo, op) are in the window (bulk literal runs bypass it)
    __device__ __forceinline__ void put(int pos, uint32_t v) const {
        ((volatile LDSA uint8_t*)b)[(pos + out.sh) & (KW - 1)] = (uint8_t)v;
    }
    __device__ __forceinline__ uint32_t get(int pos) const {
        return ((volatile const LDSA uint8_t*)b)[(pos + out.sh) & (KW - 1)];
    }
    __device__ __forceinline__ uint32_t dword(int X) const {
        return ((volatile const LDSA uint32_t*)b)[(X & (KW - 1)) >> 2];
    }
    // global <- window bytes [flushed, upto)
    __device__ __forceinline__ void flush(int upto, int lane) {
        const int fx = flushed + out.sh, ux = upto + out.sh;
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
    __device__ __forceinline__ void maybe_flush(int op, int lane) {
        if (op - flushed >= 4 * LZH_WAVE) flush(((op + out.sh) & ~3) - out.sh, lane);
    }

    // literal run in[src, src+len) -> op
    template <class W>
    __device__ __forceinline__ void literals(const W& w, const Bytes& in, int src, int op, int len, int lane) {
        if (len > 8 * LZH_WAVE) {
            // bulk: straight to global memory; the window restarts after the run
            flush(op, lane);
            copy_span(in, src, out, op, len, lane, LZH_WAVE);
            flushed = op + len;
            ringlo = op + len;
            return;
        }
        for (int base = 0; base < len; base += LZH_WAVE) {
            const int t = base + lane;
            uint32_t v;
            if (w.covers(src + base, src + base + LZH_WAVE)) v = w.lane_byte(src + t);
            else v = in.b(src + t);
            if (t < len) put(op + t, v);
            maybe_flush(op + min(base + LZH_WAVE, len), lane);
        }
    }

    // out[op + t] = out[op - off + t] for t < len (byte by byte semantics), 0 < off <= op
    __device__ __forceinline__ void match(int op, int off, int len, int lane) {
        const int src0 = op - off;
        // (reach kWin - 128: the group emitter may have written up to 127 bytes past its end)
        if (src0 >= ringlo && off <= KW - 2 * LZH_WAVE) {
            for (int base = 0; base < len; base += LZH_WAVE) {
                const int t = base + lane;
                const int s = off >= LZH_WAVE ? src0 + t : src0 + (int)((uint32_t)t % (uint32_t)off);
                const uint32_t v = get(s);
                if (t < len) put(op + t, v);
                maybe_flush(op + min(base + LZH_WAVE, len), lane);
            }
            return;
        }
        // far: the source is in global memory once every pending byte is flushed and stored
        flush(op, lane);
        for (int base = 0; base < len; base += LZH_WAVE) {
            const int t = base + lane;
            const int s = off >= LZH_WAVE ? src0 + t : src0 + (int)((uint32_t)t % (uint32_t)off);
            if (off < len && base > 0) flush(op + base, lane);   // sources in this match's output
            wait_vm();
            const uint32_t v = t < len ? out.b_sc1(s) : 0u;
            if (t < len) put(op + t, v);
        }
        maybe_flush(op + len, lane);
    }
};

typedef SinkT<kW> Sink;

}  // namespace owin

// ---------------------------------------------------------------------------------------
// One LZ4 sequence at a time with every acceptance rule of LZ4_decompress_safe (lz4.c:1707-1729,
// :1929-2151): the path for what a group does not take (255-run lengths, the last-literals
// sequence, malformed input).  Returns 0 = continue, 1 = done (last literals), < 0 = error.
namespace checked {

using owin::kW;

template <class SinkType>
__device__ __forceinline__ int lz4_one(const Bytes& in, int cs, SinkType& O, Win& w, int cap, int& ip, int& op,
                                       int lane, int prefix = 0) {
    if (ip >= cs) return -ip - 1;
    w.ensure(ip, lane);
    const uint32_t tok = w.byte(ip++);
    int lit = (int)(tok >> 4);
    if (lit == 15) {
        if (ip >= cs - 15) return -ip - 1;
        for (int it = 0; it <= cs; it++) {
            w.ensure(ip, lane);
            const uint32_t s = w.byte(ip++);
            lit += (int)s;
            if (ip >= cs - 15 || s != 255) break;
        }
    }
    if (op + lit > cap - 12 || ip + lit > cs - 8) {
        if (ip + lit != cs || op + lit > cap) return -ip - 1;
        O.literals(w, in, ip, op, lit, lane);
        op += lit;
        return 1;
    }
    O.literals(w, in, ip, op, lit, lane);
    ip += lit;
    op += lit;
    w.ensure(ip, lane);
    const int off = (int)(w.byte(ip) | (w.byte(ip + 1) << 8));
    ip += 2;
    int ml = (int)(tok & 15u);
    if (ml == 15) {
        for (int it = 0; it <= cs; it++) {
            w.ensure(ip, lane);
            const uint32_t s = w.byte(ip++);
            ml += (int)s;
            if (ip >= cs - 4) return -ip - 1;
            if (s != 255) break;
        }
    }
    ml += 4;
    if (off > op + prefix) return -ip - 1;   // (prefix: earlier output of a linked frame, lz4.c:2404-2416)
    if (op + ml > cap - 5) return -ip - 1;
    if (off == 0) {
        for (int base = 0; base < ml; base += LZH_WAVE) {
            if (base + lane < ml) O.put(op + base + lane, 0);
            O.maybe_flush(op + min(base + LZH_WAVE, ml), lane);
        }
    } else {
        O.match(op, off, ml, lane);
    }
    op += ml;
    return 0;
}

}  // namespace checked

// ---------------------------------------------------------------------------------------
// Groups resolved lane-parallel.  Every lane parses "a sequence at ip + lane" in full (token, one
// literal-length byte, offset, one match-length byte) from the register window; binary lifting
// over the per-lane next-token links (chain_members) picks the real chain;
// the reference acceptance rules are checked per member lane against a DPP prefix sum of the
// output lengths, and the chain is cut before the first member that fails them (it, the last
// sequence and sequences with 255-run lengths go through the checked path).  Output bytes are
// assembled one per lane per pass: the owning sequence is found from per-pass start marks in
// LDS, literal bytes come from the register window, match bytes from the LDS output window (or
// global memory for far sources) in dependency rounds.
namespace groups {

using owin::kW;

__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return x;
}

// Output byte ob (group-relative) from its owner's fields, precomputed per member so that a byte
// costs adds and compares only: lend = the owner's literal end (group-relative), lsb = stream
// position of its literal byte at ob = lsb + ob, msrc = absolute output position of its match
// source at ob = msrc + ob (byte-by-byte semantics; overlapping copies take the period form).
// done = final now (not an unresolved in-pass source); far = source only in global memory.
template <class W, class SinkType>
__device__ __forceinline__ uint32_t owned_byte(const W& w, const SinkType& O, int op, int pbase, int thr, int ob,
                                               int total, int lend, int lsb, int msrc, int offk, int& src,
                                               uint64_t& done, uint64_t& far) {
    // (lane masks from single-compare ballots: a ballot of a compound bool goes through a VGPR)
    const uint64_t il = ballot(ob < lend), act = ballot(ob < total);
    const bool is_lit = lane_on(il);
    const uint32_t lb = w.lane_byte(lsb + (is_lit ? ob : lend - 1));
    src = msrc + ob;
    const uint64_t ov = ballot(ob >= lend + offk) & ~il;
    if (ov & act) {                                                // overlapping copy: period offk
        const int md = (int)((uint32_t)(ob - lend) % (uint32_t)max(offk, 1));
        src = lane_on(ov) ? op + lend - offk + md : src;
    }
    const uint32_t g = O.get(src);
    const uint64_t near = ballot(src >= O.ringlo) & ballot(src >= thr) & ~il;
    const uint64_t inpass = ballot(src >= pbase) & ~il;
    done = il | (near & ~inpass);
    far = act & ~il & ~near;
    return is_lit ? lb : g;
}

// The part of a 128-byte pass after its far reads are issued (their data are used here first):
// store the bytes, resolve in-pass sources in dependency rounds, flush.
struct Tail {
    uint64_t far0, far1, done0, done1;   // (lane masks)
    uint32_t v0, v1, g0, g1;
    int src0, src1, ob0, ob1, pbase, op, total;
};

template <class SinkType>
__device__ __forceinline__ void pass_tail(SinkType& O, Tail& t, int lane) {
    constexpr int kP = 2 * LZH_WAVE;
    const uint32_t v0 = lane_on(t.far0) ? t.g0 : t.v0, v1 = lane_on(t.far1) ? t.g1 : t.v1;
    const int op = t.op, pbase = t.pbase, ob0 = t.ob0, ob1 = t.ob1, src0 = t.src0, src1 = t.src1;
    // (bytes past the group's end land in window slots at most 127 bytes past it, which no
    // later reader takes as near: the next group's threshold, SinkT::match's kWin - 128 reach)
    O.put(op + ob0, v0);
    O.put(op + ob1, v1);
    // in-pass sources: rounds until every byte read a finished source
    uint64_t dm0 = t.done0 | t.far0 | ballot(ob0 >= t.total), dm1 = t.done1 | t.far1 | ballot(ob1 >= t.total);
    uint32_t w0 = v0, w1 = v1;
    for (int r = 0; r < kP && (~dm0 | ~dm1); r++) {
        DST(4, 1);
        const int s0 = src0 - pbase, s1 = src1 - pbase;
        // (the lanes that read a finished source, as masks: one compare per ballot -- a ballot of the compound
        // bool goes through a VGPR)
        const uint64_t rm0 = ballot((((s0 & 1 ? dm1 : dm0) >> ((s0 >> 1) & 63)) & 1ull) != 0ull) & ~dm0;
        const uint64_t rm1 = ballot((((s1 & 1 ? dm1 : dm0) >> ((s1 >> 1) & 63)) & 1ull) != 0ull) & ~dm1;
        const bool rd0 = lane_on(rm0), rd1 = lane_on(rm1);
        const uint32_t q0 = O.get(src0), q1 = O.get(src1);
        w0 = rd0 ? q0 : w0;
        w1 = rd1 ? q1 : w1;
        O.put(op + ob0, w0);
        O.put(op + ob1, w1);
        dm0 |= rm0;
        dm1 |= rm1;
    }
    O.maybe_flush(min(pbase + kP, op + t.total), lane);
}

// Two output bytes per lane per pass (128-byte passes): a byte pair has at most two owners (the
// member owning its first byte, and one starting at its second), so each pass gathers two sets of
// member fields instead of one per 64 bytes.  Marks: 128 bytes + 64 bytes of scratch.
template <class W, class SinkType>
__device__ __forceinline__ void emit_group(const W& w, SinkType& O, LDSA uint8_t* mark, int ip, int op,
                                           int total, uint64_t keep, int excl, uint32_t pA, uint32_t lrel,
                                           int off, int lane) {
    constexpr int kP = 2 * LZH_WAVE;
    const bool kmem = lane_on(keep);
    int carry = 63 - __builtin_clzll(keep);                      // (pass 0 always has a start at 0)
    // per member: literal end, literal stream base, match source base (see owned_byte)
    const int m_lend = excl + (int)(pA & 0xffffu);
    const int m_lsb = ip + (int)lrel - excl;
    const int m_msrc = op - off;
    const uint64_t below = (1ull << lane) - 1ull;
    Tail t;
    for (int pb = 0; pb < total; pb += kP) {
        DMARK(10);
        ((volatile LDSA uint16_t*)mark)[lane] = 0xffffu;
        wave_lds_fence();
        const bool mine = kmem && excl >= pb && excl < pb + kP;
        mark[mine ? excl - pb : kP + lane] = (uint8_t)lane;
        wave_lds_fence();
        const uint32_t mm = ((volatile LDSA uint16_t*)mark)[lane];
        const uint32_t m0 = mm & 0xffu, m1 = mm >> 8;
        // owner of the lane's first byte: its own mark, else the last mark of an earlier lane
        const uint64_t lt_ = ballot(mm != 0xffffu) & below;
        const int js = lt_ ? 63 - __builtin_clzll(lt_) : lane;
        const uint32_t mj = lane_gather(mm, js);
        const int prevk = lt_ ? (int)((mj >> 8) != 0xffu ? (mj >> 8) : (mj & 0xffu)) : carry;
        const int k0 = m0 != 0xffu ? (int)m0 : prevk;
        const int k1 = m1 != 0xffu ? (int)m1 : k0;
        carry = rdlanei(k1, 63);
        const int le0 = (int)lane_gather((uint32_t)m_lend, k0), ls0 = (int)lane_gather((uint32_t)m_lsb, k0),
                  ms0 = (int)lane_gather((uint32_t)m_msrc, k0), of0 = (int)lane_gather((uint32_t)off, k0);
        int le1 = le0, ls1 = ls0, ms1 = ms0, of1 = of0;
        DST(2, 1);
        if (ballot(k1 != k0)) {
            DST(3, 1);
            le1 = (int)lane_gather((uint32_t)m_lend, k1);
            ls1 = (int)lane_gather((uint32_t)m_lsb, k1);
            ms1 = (int)lane_gather((uint32_t)m_msrc, k1);
            of1 = (int)lane_gather((uint32_t)off, k1);
        }
        DMARK(11);
        const int pbase = op + pb;
        const int thr = pbase + kP - SinkType::kWin;               // sources below: overwritten in the window
        const int ob0 = pb + 2 * lane, ob1 = ob0 + 1;
        int src0, src1;
        uint64_t done0, done1, far0, far1;
        const uint32_t v0 = owned_byte(w, O, op, pbase, thr, ob0, total, le0, ls0, ms0, of0, src0, done0, far0);
        const uint32_t v1 = owned_byte(w, O, op, pbase, thr, ob1, total, le1, ls1, ms1, of1, src1, done1, far1);
        DMARK(12);
        t.g0 = t.g1 = 0;
        const bool anyfar = (far0 | far1) != 0;
        if (anyfar) {   // far sources were flushed long ago: their stores must be done
            DST(5, 1);
            wait_vm();
            t.g0 = O.out.b_sc1(lane_on(far0) ? src0 : 0);
            t.g1 = O.out.b_sc1(lane_on(far1) ? src1 : 0);
        }
        t.far0 = far0; t.far1 = far1; t.done0 = done0; t.done1 = done1;
        t.v0 = v0; t.v1 = v1; t.src0 = src0; t.src1 = src1; t.ob0 = ob0; t.ob1 = ob1;
        t.pbase = pbase; t.op = op; t.total = total;
        DMARK(13);
        pass_tail(O, t, lane);
        DMARK(14);
    }
}

// Lanes on the chain that starts at lane 0 and follows `link` (next lane, strictly increasing;
// >= 64 = leaves the group, 255 = the lane itself is not taken), by binary lifting: jump tables
// J_k = link^(2^k) through ds_bpermute, then every lane lifts from lane 0 to the furthest chain
// lane <= itself.  No scalar walk (the decoder is scalar-issue bound).
__device__ __forceinline__ uint64_t chain_members(int link, int lane) {
    // (every member takes >= 2 stream bytes -- a snappy literal tag + 1 byte or a COPY_1, LZ4 >= 3 --
    // so a chain from lane 0 has at most 32 members: jumps of 1..16 reach every one of them)
    const int J0 = min(link, LZH_WAVE);
    const int J1 = J0 < LZH_WAVE ? (int)lane_gather((uint32_t)J0, J0) : LZH_WAVE;
    const int J2 = J1 < LZH_WAVE ? (int)lane_gather((uint32_t)J1, J1) : LZH_WAVE;
    const int J3 = J2 < LZH_WAVE ? (int)lane_gather((uint32_t)J2, J2) : LZH_WAVE;
    const int J4 = J3 < LZH_WAVE ? (int)lane_gather((uint32_t)J3, J3) : LZH_WAVE;
    int x = 0, y;
    y = (int)lane_gather((uint32_t)J4, x); x = y <= lane ? y : x;
    y = (int)lane_gather((uint32_t)J3, x); x = y <= lane ? y : x;
    y = (int)lane_gather((uint32_t)J2, x); x = y <= lane ? y : x;
    y = (int)lane_gather((uint32_t)J1, x); x = y <= lane ? y : x;
    y = (int)lane_gather((uint32_t)J0, x); x = y <= lane ? y : x;
    return ballot(x == lane) & ballot(link != 255);   // (single compares: no VGPR round trip)
}

template <class SinkType>
__device__ int lz4_decode(const Bytes& in, int cs, SinkType& O, LDSA uint8_t* mark, LDSA uint8_t* ring, int cap,
                          int lane, int prefix = 0) {
    if (cap == 0) return (cs == 1 && in.b(0) == 0) ? 0 : -1;
    if (cs <= 0) return -1;
    Win w;
    w.bind(in, ring);
    w.load(0, lane);
    int ip = 0, op = 0;
    for (int guard = 0; guard <= cs; guard++) {
        DCLK(t0);
        DMARK(0);
        ip = unii(ip); op = unii(op);
        O.flushed = unii(O.flushed); O.ringlo = unii(O.ringlo);
        if (!w.covers(ip, ip + 2 * LZH_WAVE)) w.load(ip, lane);
        // ---- every lane parses a whole sequence at x = ip + lane (lz4.c:1707-1729, :1929-2151)
        const int x = ip + lane;
        const uint32_t tw = w.lane_word(x);
        const int ln = (int)((tw >> 4) & 15u), mc = (int)(tw & 15u), b1 = (int)((tw >> 8) & 255u);
        const int lit = ln == 15 ? 15 + b1 : ln;
        const int p1 = x + 1 + (ln == 15 ? 1 : 0);                // first literal byte
        const int po = p1 + lit;                                    // offset bytes
        const bool inwin = w.covers(po, po + 4);
        const uint32_t ow = w.lane_word(inwin ? po : x);
        const int off = (int)(ow & 0xffffu), b2 = (int)((ow >> 16) & 255u);
        const int ml = mc == 15 ? 19 + b2 : mc + 4;
        const int pe = po + 2 + (mc == 15 ? 1 : 0);                 // next token
        const bool cplx = !inwin || (ln == 15 && b1 == 255) || (mc == 15 && b2 == 255);
        const int link = cplx ? 255 : pe - ip;
        // ---- the real chain from lane 0
        DMARK(1);
        const uint64_t M = chain_members(link, lane);
        DMARK(2);
        // ---- acceptance rules per member (as lz4_one); the chain ends before the first failure
        const bool mem = lane_on(M);
        const int L = mem ? lit + ml : 0;
        const int incl = wave_incl_scan(L);
        const int excl = incl - L;
        const int opm = op + excl + lit;
        // (the failing members as a mask of single-compare ballots: a ballot of the compound bool goes through a VGPR)
        const uint64_t badm = M & (ballot(x >= cs) | (ballot(ln == 15) & ballot(x + 1 >= cs - 15)) | ballot(opm > cap - 12) |
                                   ballot(p1 + lit > cs - 8) | (ballot(mc == 15) & ballot(po + 3 >= cs - 4)) |
                                   ballot(off == 0) | ballot(off > opm + prefix) | ballot(opm + ml > cap - 5));
        const uint64_t keep = badm ? (M & ((1ull << __builtin_ctzll(badm)) - 1ull)) : M;
        if (!keep) {
            const int r = checked::lz4_one(in, cs, O, w, cap, ip, op, lane, prefix);
            DST(6, 1);
#if LZH_DEC_STATS
            DST(10, __builtin_amdgcn_s_memtime() - t0);
#endif
            if (r < 0) return r;
            if (r == 1) break;
            continue;
        }
        const int lastk = 63 - __builtin_clzll(keep);
        const int total = rdlanei(incl, lastk);
        const int ip_next = ip + rdlanei(pe - ip, lastk);
        DCLK(t1);
        DMARK(3);
        emit_group(w, O, mark, ip, op, total, keep, excl, (uint32_t)lit | ((uint32_t)ml << 16), (uint32_t)(p1 - ip),
                   off, lane);
#if LZH_DEC_STATS
        DCLK(t2);
        DST(0, 1);
        DST(1, __builtin_popcountll(keep));
        DST(7, total);
        DST(8, t1 - t0);
        DST(9, t2 - t1);
#endif
        op += total;
        ip = ip_next;
    }
    return op;
}


// snappy tags a group at a time (same scheme): every lane parses a tag at ip + lane (literal with
// at most one length byte, COPY_1/2/4), the walk follows the next-tag links, the acceptance rules
// of snappy_decode below (snappy.cc:848-952) are checked per member against the prefix sum, and
// the group is cut before the first failure (which, like 2..4-byte literal lengths, runs through
// the checked per-tag path).
// (nohdr: a fragment of a stream -- its tags without the varint, decoding exactly cap bytes; see
// lzh_snappy_split_kernel)
template <class SinkType>
__device__ int snappy_decode(const Bytes& in, int cs, SinkType& O, LDSA uint8_t* mark, LDSA uint8_t* ring, int cap,
                             int lane, bool nohdr = false) {
    Win w;
    w.bind(in, ring);
    w.load(0, lane);
    int ip = 0;
    uint32_t ulen = nohdr ? (uint32_t)cap : 0u;
    for (int shift = 0; !nohdr; shift += 7) {
        if (ip >= cs || shift >= 32) return -1;
        const uint32_t c = w.byte(ip++);
        const uint32_t val = c & 0x7fu;
        if (shift == 28 && val > 15) return -1;
        ulen |= val << shift;
        if (c < 128) break;
    }
    if (ulen > (uint32_t)cap) return -1;
    const int ul = (int)ulen;
    int op = 0;
    for (int guard = 0; guard <= cs && ip < cs; guard++) {
        ip = unii(ip); op = unii(op);
        O.flushed = unii(O.flushed); O.ringlo = unii(O.ringlo);
        if (!w.covers(ip, ip + 2 * LZH_WAVE)) w.load(ip, lane);
        const int x = ip + lane;
        const uint32_t tw = w.lane_word(x);
        const uint32_t c = tw & 0xffu, kind = c & 3u;
        int len, lit, nx, off = 0, p1 = x + 1;
        bool cplx = false, okr = true;
        if (kind == 0) {
            const int l6 = (int)(c >> 2) + 1;
            const bool one = l6 == 61;                              // one length byte
            cplx = l6 > 61;
            len = one ? (int)((tw >> 8) & 0xffu) + 1 : l6;
            p1 = x + 1 + (one ? 1 : 0);
            lit = len;
            nx = p1 + len;
            okr = (!one || x + 2 <= cs) && p1 + len <= cs;
        } else {
            const int extra = kind == 1 ? 1 : (kind == 2 ? 2 : 4);
            const uint32_t tw2 = w.lane_word(x + 1);
            if (kind == 1) {
                len = (int)((c >> 2) & 7u) + 4;
                off = (int)(((c >> 5) << 8) | ((tw >> 8) & 0xffu));
            } else {
                len = (int)(c >> 2) + 1;
                off = kind == 2 ? (int)((tw >> 8) & 0xffffu) : (int)tw2;
            }
            lit = 0;
            nx = x + 1 + extra;
            okr = nx <= cs && off > 0 && (uint32_t)off <= (uint32_t)cap;
        }
        const bool inwin = w.covers(x, nx + 4);
        // link: next tag lane; 255 = not parsed here; 254 = the stream ends after this tag
        const int link = (cplx || !inwin || x >= cs) ? 255 : (nx >= cs ? 254 : nx - ip);
        const uint64_t M = chain_members(link, lane);
        const bool mem = lane_on(M);
        const int L = mem ? len : 0;
        const int incl = wave_incl_scan(L);
        const int excl = incl - L;
        const int opm = op + excl;
        const uint64_t badm = M & (ballot(x >= cs) | ~ballot(okr) | ballot(opm + len > ul) |
                                   (ballot(kind != 0) & ballot(off > opm)));   // (single-compare ballots)
        const uint64_t keep = badm ? (M & ((1ull << __builtin_ctzll(badm)) - 1ull)) : M;
        if (!keep) {
            // one tag through the checked path (snappy.cc:848-952 rules)
            const uint32_t cc = w.byte(ip++);
            const uint32_t kk = cc & 3u;
            if (kk == 0) {
                int ln = (int)(cc >> 2) + 1;
                if (ln > 60) {
                    const int nb = ln - 60;
                    if (ip + nb > cs) return -1;
                    uint32_t v = 0;
                    for (int i = 0; i < nb; i++) v |= w.byte(ip + i) << (8 * i);
                    ln = (int)v + 1;
                    if (v >= 0x7fffffffu) return -1;
                    ip += nb;
                }
                if ((int64_t)ip + ln > cs || (int64_t)op + ln > ul) return -1;
                O.literals(w, in, ip, op, ln, lane);
                ip += ln;
                op += ln;
            } else {
                const int extra = kk == 1 ? 1 : (kk == 2 ? 2 : 4);
                if (ip + extra > cs) return -1;
                int ln;
                uint32_t of;
                if (kk == 1) {
                    ln = (int)((cc >> 2) & 7u) + 4;
                    of = ((cc >> 5) << 8) | w.byte(ip);
                } else {
                    ln = (int)(cc >> 2) + 1;
                    of = 0;
                    for (int i = 0; i < extra; i++) of |= w.byte(ip + i) << (8 * i);
                }
                ip += extra;
                if (of == 0 || of > (uint32_t)op || op + ln > ul) return -1;
                O.match(op, (int)of, ln, lane);
                op += ln;
            }
            continue;
        }
        const int lastk = 63 - __builtin_clzll(keep);
        const int total = rdlanei(incl, lastk);
        const int ip_next = ip + rdlanei(nx - ip, lastk);
        emit_group(w, O, mark, ip, op, total, keep, excl, (uint32_t)lit | ((uint32_t)(len - lit) << 16),
                   (uint32_t)(p1 - ip), off, lane);
        op += total;
        ip = ip_next;
    }
    return op == ul ? op : -1;
}

}  // namespace groups

// One chunk (or framed block) per wave; KW = bytes of the LDS output window.  The window sets the
// share of match sources read from the LDS instead of the flushed output in global memory, and the
// LDS per wave (hence waves per CU): lzh_launch_decompress picks the largest window whose occupancy
// still holds every chunk of the launch at once.
template <int KW>
__device__ __forceinline__ void decompress_chunk(LDSA uint8_t* win, int codec, const uint8_t* packed,
                                                 uint64_t packed_readable, const uint64_t* offsets,
                                                 const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size,
                                                 uint8_t* out, int32_t* status, uint32_t chunk0, const uint32_t* desc) {
    const int lane = threadIdx.x;
    const uint64_t chunk = (uint64_t)blockIdx.x + chunk0;
    uint64_t ooff, ioff;
    int part, cs;
    bool raw, nohdr = false;
    if (desc) {   // framed layouts: one 32-byte block descriptor each (frame_hip.hip FrameDesc)
        const uint32_t* d = desc + 8 * chunk;
        ioff = (uint64_t)uni(d[1]) << 32 | uni(d[0]);
        ooff = (uint64_t)uni(d[3]) << 32 | uni(d[2]);
        cs = (int)uni(d[4]);
        part = (int)uni(d[5]);
        const uint32_t fl = uni(d[6]);
        raw = (fl & 1u) != 0;
        nohdr = (fl & 8u) != 0;                 // a snappy fragment (lzh_snappy_split_kernel)
        if (fl & 22u) return;                   // a linked frame's block: lzh_decompress_linked_kernel; 16: skip
        if (part == 0) { if (lane == 0) status[chunk] = 0; return; }   // unused slot
    } else {
        ooff = chunk * chunk_size;
        if (ooff >= n_total) return;
        part = (int)min(chunk_size, n_total - ooff);
        ioff = offsets[chunk];
        cs = (int)csizes[chunk];
        raw = cs == part || codec == 2;
    }
#if LZH_DEC_STATS
    if (lane < 16) g_dst[lane] = 0;
    DCLK(tk0);
#endif
    const uint64_t readable = ioff < packed_readable ? min<uint64_t>(packed_readable - ioff, (uint64_t)cs + 16) : 0;
    Bytes rin, rout;
    rin.init(packed + ioff, readable);
    rout.init(out + ooff, (uint64_t)part);
    int r;
    if (raw) {
        copy_raw(rin, rout, part, lane);
        r = part;
    } else {
        owin::SinkT<KW> O{win, rout, 0, 0};
        LDSA uint8_t* mark = win + KW;
        LDSA uint8_t* ring = mark + 3 * LZH_WAVE;
        r = codec == 0 ? groups::lz4_decode(rin, cs, O, mark, ring, part, lane)
                       : groups::snappy_decode(rin, cs, O, mark, ring, part, lane, nohdr);
        if (r > 0) O.flush(r, lane);
    }
    if (lane == 0) status[chunk] = r;
#if LZH_DEC_STATS
    DST(11, 1);
    DST(12, __builtin_amdgcn_s_memtime() - tk0);
    if (lane < 16) atomicAdd(&lzh_dec_stats_buf[lane], g_dst[lane]);
#endif
}

// output window | start marks | input ring
#define LZH_DEC_KERNEL(NAME, KW)                                                                            \
    extern "C" __global__ void __launch_bounds__(64)                                                       \
    NAME(int codec, const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,              \
         const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint8_t* out, int32_t* status,     \
         uint32_t chunk0, const uint32_t* desc) {                                                          \
        __shared__ __attribute__((aligned(16))) uint8_t win[KW + 3 * LZH_WAVE + kRingBytes];              \
        decompress_chunk<KW>((LDSA uint8_t*)win, codec, packed, packed_readable, offsets, csizes, n_total,  \
                             chunk_size, out, status, chunk0, desc);                                       \
    }
LZH_DEC_KERNEL(lzh_decompress_v2_kernel, owin::kW)
LZH_DEC_KERNEL(lzh_decompress_w8k_kernel, 8192)
LZH_DEC_KERNEL(lzh_decompress_w16k_kernel, 16384)
#undef LZH_DEC_KERNEL

// LZ4 frames with linked blocks (frame_hip.hip marks their descriptors: flags 2 = a frame's first
// block, pad = its block count; 4 = a later block): one wave per frame decodes the blocks in order,
// each with the frame's output before it as its prefix (LZ4F_updateDict's prefix mode,
// lz4frame.c:1290-1306; LZ4_decompress_safe_usingDict, lz4.c:2404-2416): a match may reach back
// into earlier blocks (read from global memory, the window starts empty per block), and the offset
// check fails only past the frame's start.  Waves of other descriptors exit at once.
extern "C" __global__ void __launch_bounds__(64)
lzh_decompress_linked_kernel(const uint8_t* packed, uint64_t packed_readable, uint8_t* out, int32_t* status,
                             const uint32_t* desc) {
    __shared__ __attribute__((aligned(16))) uint8_t win[owin::kW + 3 * LZH_WAVE + kRingBytes];
    const int lane = threadIdx.x;
    const uint64_t chunk = blockIdx.x;
    const uint32_t* d0 = desc + 8 * chunk;
    if (!(uni(d0[6]) & 2u)) return;
    const uint32_t nlink = uni(d0[7]);
    const uint64_t foff = (uint64_t)uni(d0[3]) << 32 | uni(d0[2]);   // the frame's output start
    for (uint32_t bi = 0; bi < nlink; bi++) {
        const uint32_t* d = desc + 8 * (chunk + bi);
        const uint64_t ioff = (uint64_t)uni(d[1]) << 32 | uni(d[0]);
        const uint64_t ooff = (uint64_t)uni(d[3]) << 32 | uni(d[2]);
        const int cs = (int)uni(d[4]), part = (int)uni(d[5]);
        const bool raw = (uni(d[6]) & 1u) != 0;
        wait_vm();   // (the previous block's output stores are done before its bytes are read back)
        const int prefix = (int)(ooff - foff);
        const uint64_t readable = ioff < packed_readable ? min<uint64_t>(packed_readable - ioff, (uint64_t)cs + 16) : 0;
        Bytes rin, rout;
        rin.init(packed + ioff, readable);
        rout.init(out + foff, (uint64_t)prefix + part);
        rout.sh += prefix;                    // (block positions; earlier output at negative ones)
        int r;
        if (raw) {
            copy_raw(rin, rout, part, lane);
            r = part;
        } else {
            owin::Sink O{(LDSA uint8_t*)win, rout, 0, 0};
            LDSA uint8_t* mark = (LDSA uint8_t*)win + owin::kW;
            LDSA uint8_t* ring = mark + 3 * LZH_WAVE;
            r = groups::lz4_decode(rin, cs, O, mark, ring, part, lane, prefix);
            if (r > 0) O.flush(r, lane);
        }
        if (lane == 0) status[chunk + bi] = r;
        if (r < 0) {   // the frame is bad: its remaining blocks are not decoded
            for (uint32_t bj = bi + 1 + (uint32_t)lane; bj < nlink; bj += LZH_WAVE) status[chunk + bj] = -1;
            break;
        }
    }
}

// ---------------------------------------------------------------------------------------
// Snappy chunks of more than one 64 KiB fragment, decoded a fragment per wave.  The reference
// compressor compresses every 64 KiB fragment of its input on its own (snappy.cc:1042-1072: a fresh
// table per fragment, candidates only inside it), so the tags of a stream it wrote start anew at every
// multiple of 64 KiB of output and no copy reaches into an earlier fragment.  lzh_snappy_split_kernel
// walks a chunk's tags (one wave per chunk: every lane parses the tag at ip + lane, a scalar walk
// follows the next-tag links and sums the output lengths) and records the tag that starts each
// fragment; the fragments then decode in parallel as headerless streams of exactly their size
// (descriptor flag 8).  A chunk that the walk does not split cleanly (a tag across a fragment start, a
// varint that is not the chunk's size, a stored chunk, a walk off the stream) or any fragment of which
// fails (a copy into an earlier fragment is valid snappy, just not what the reference writes) is
// decoded whole by the serial decoder afterwards, so every verdict and every byte of such a chunk is
// the serial decoder's.  An accepted split decodes the same tags in the same order as the serial
// decoder: the fragments partition the chunk's tag sequence, each ends exactly at its share of the
// stream and of the output, and a copy accepted inside a fragment is accepted in the chunk.
namespace snsplit {
constexpr int kFragLog = 16;
constexpr uint32_t kMaxFrags = 64;   // chunks of up to 4 MiB (larger ones decode whole)
constexpr uint32_t kMinFrags = 8;    // (by default; see lzh_snappy_split_temp)
__host__ __device__ inline uint32_t frags(uint64_t chunk_size) { return (uint32_t)((chunk_size + 65535) >> kFragLog); }
}

extern "C" __global__ void __launch_bounds__(64)
lzh_snappy_split_kernel(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                        const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint32_t F, uint32_t* desc,
                        uint32_t* cflag) {
    using namespace snsplit;
    __shared__ __attribute__((aligned(16))) uint8_t ring[kRingBytes];
    __shared__ uint32_t bnd[kMaxFrags + 1];
    const int lane = threadIdx.x;
    const uint64_t chunk = blockIdx.x;
    const uint64_t ooff = chunk * chunk_size;
    if (ooff >= n_total) return;
    const int part = (int)min(chunk_size, n_total - ooff);
    const uint64_t ioff = offsets[chunk];
    const int cs = (int)csizes[chunk];
    const int nf = (part + (1 << kFragLog) - 1) >> kFragLog;
    bool ok = cs != part && nf > 1 && nf <= (int)F && F <= kMaxFrags;
    int ip = 0, op = 0, nb = 0;
    if (ok) {   // (a uniform walk: ip, op, nb in scalar registers)
        const uint64_t readable = ioff < packed_readable ? min<uint64_t>(packed_readable - ioff, (uint64_t)cs + 16) : 0;
        Bytes rin;
        rin.init(packed + ioff, readable);
        Win w;
        w.bind(rin, (LDSA uint8_t*)ring);
        w.load(0, lane);
        uint32_t ulen = 0;
        for (int shift = 0;; shift += 7) {   // varint32 uncompressed length (snappy.cc:1319-1331)
            if (ip >= cs || shift >= 32) { ok = false; break; }
            const uint32_t c = w.byte(ip++);
            ulen |= (c & 0x7fu) << shift;
            if (c < 128) break;
        }
        ok = ok && ulen == (uint32_t)part;
        if (lane == 0) bnd[0] = (uint32_t)ip;   // fragment 0 starts after the varint
        nb = 1;
        for (int guard = 0; ok && ip < cs && guard <= cs; guard++) {
            ip = unii(ip); op = unii(op); nb = unii(nb);
            if (!w.covers(ip, ip + 2 * LZH_WAVE)) w.load(ip, lane);
            // the tag at x = ip + lane: its stream length and output length (snappy.cc:848-952)
            const int x = ip + lane;
            const uint32_t tw = w.lane_word(x);
            const uint32_t c = tw & 0xffu, kind = c & 3u;
            uint32_t tw2 = 0;                       // (a 4-byte literal length reaches byte x + 4)
            if (ballot(c == 0xfcu)) tw2 = w.lane_word(x + 1);
            uint32_t len, sl;                       // output bytes, stream bytes after the tag byte
            if (kind == 0) {
                const uint32_t l6 = (c >> 2) + 1u;
                const uint32_t eb = l6 > 60u ? l6 - 60u : 0u;   // 1..4 length bytes
                const uint32_t v = eb == 4u ? tw2 : ((tw >> 8) & ((1u << (8u * eb)) - 1u));
                const uint32_t l = eb ? (v >= 0x00ffffffu ? 0x00ffffffu : v + 1u) : l6;   // (beyond any chunk)
                len = l;
                sl = eb + l;
            } else {
                len = kind == 1 ? ((c >> 2) & 7u) + 4u : (c >> 2) + 1u;
                sl = kind == 1 ? 1u : (kind == 2 ? 2u : 4u);
            }
            const int adv_l = lane + 1 + (int)sl;              // next tag, from ip (> lane)
            // the chain from lane 0 (binary lifting, as the decoder's groups); lanes at or past the
            // stream's end are not tags
            // (255 is chain_members' "not a tag": a real link that leaves the window is any value >= 64)
            const int link = x >= cs ? 255 : min(adv_l, 254);
            const uint64_t M = groups::chain_members(link, lane);
            const bool mem = lane_on(M);
            const int L = mem ? (int)len : 0;
            const int incl = groups::wave_incl_scan(L);
            const int start = op + incl - L;                   // a member's first output byte
            // a member starting on a multiple of 64 KiB starts that fragment
            const bool fb = mem && start > 0 && (start & ((1 << kFragLog) - 1)) == 0 && (start >> kFragLog) < nf;
            if (fb) bnd[start >> kFragLog] = (uint32_t)x;
            nb += __builtin_popcountll(ballot(fb));
            const int lastk = 63 - __builtin_clzll(M | 1ull);
            op += rdlanei(incl, lastk);
            ip += rdlanei(adv_l, lastk);
            if (op > part) ok = false;
        }
        ok = ok && ip == cs && op == part && nb == nf;
    }
    wave_lds_fence();
    uint32_t* D = desc + chunk * (uint64_t)F * 8;
    for (int j = lane; j < (int)F; j += LZH_WAVE) {   // fragment j; unused slots decode nothing (ds = 0)
        uint32_t a = 0, e = 0, ds = 0;
        if (ok && j < nf) {
            a = bnd[j];
            e = j + 1 < nf ? bnd[j + 1] : (uint32_t)cs;
            ds = (uint32_t)min(1 << kFragLog, part - (j << kFragLog));
        }
        const uint64_t src = ioff + a, dst = ooff + ((uint64_t)j << kFragLog);
        uint32_t* d = D + 8 * j;
        d[0] = (uint32_t)src; d[1] = (uint32_t)(src >> 32);
        d[2] = (uint32_t)dst; d[3] = (uint32_t)(dst >> 32);
        d[4] = e - a; d[5] = ds; d[6] = 8u; d[7] = 0u;
    }
    if (lane == 0) cflag[chunk] = ok ? 0u : 1u;
}

// chunks finished by fragments since the last reset (tests: lzh_debug_snappy_split_done)
__device__ unsigned long long lzh_snsplit_done;

// per chunk: split and every fragment decoded exactly its size -> the chunk's status; else a whole-chunk
// descriptor for the serial pass (flag 16 = skip for the others)
extern "C" __global__ void __launch_bounds__(256)
lzh_snappy_join_kernel(const uint64_t* offsets, const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size,
                       uint32_t F, const uint32_t* desc, const int32_t* fstat, const uint32_t* cflag, uint32_t* sdesc,
                       int32_t* status, uint32_t nchunks) {
    const uint64_t c = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (c >= nchunks) return;
    const uint64_t ooff = c * chunk_size;
    const uint32_t part = (uint32_t)min(chunk_size, n_total - ooff);
    bool whole = cflag[c] != 0u;
    for (uint32_t j = 0; !whole && j < F; j++) {
        const uint32_t ds = desc[(c * F + j) * 8 + 5];
        if (ds && fstat[c * F + j] != (int32_t)ds) whole = true;
    }
    uint32_t* S = sdesc + c * 8;
    if (whole) {
        const uint64_t io = offsets[c];
        const uint32_t cs = csizes[c];
        S[0] = (uint32_t)io; S[1] = (uint32_t)(io >> 32);
        S[2] = (uint32_t)ooff; S[3] = (uint32_t)(ooff >> 32);
        S[4] = cs; S[5] = part; S[6] = cs == part ? 1u : 0u; S[7] = 0u;
    } else {
        S[0] = S[1] = S[2] = S[3] = S[4] = S[5] = S[7] = 0u;
        S[6] = 16u;
        status[c] = (int32_t)part;
        atomicAdd(&lzh_snsplit_done, 1ull);
    }
}

#if LZH_DEC_STATS
extern "C" int lzh_debug_dec_stats(unsigned long long* host, int reset) {
    if (reset) {
        unsigned long long z[16] = {};
        return hipMemcpyToSymbol(HIP_SYMBOL(lzh_dec_stats_buf), z, sizeof(z)) == hipSuccess ? 0 : -1;
    }
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(lzh_dec_stats_buf), 16 * sizeof(unsigned long long)) == hipSuccess ? 0 : -1;
}
#endif

// ---------------------------------------------------------------------------------------
// zstd frames (RFC 8878), the decode side of lzbench's zstd rows (compressors.cpp:1767-1773:
// ZSTD_decompressDCtx of one frame per chunk).  Reference decoder: zstd 1.5.2
//   frame / blocks       zstd/lib/decompress/zstd_decompress.c (ZSTD_decompressFrame)
//   literals, sequences  zstd/lib/decompress/zstd_decompress_block.c (ZSTD_decodeLiteralsBlock,
//                        ZSTD_decodeSeqHeaders, ZSTD_buildFSETable, ZSTD_decodeSequence,
//                        ZSTD_decompressSequences_body)
//   Huffman              zstd/lib/decompress/huf_decompress.c (HUF_readDTableX1, 1X1 / 4X1 streams;
//                        the 1X2 / 4X2 acceptance rules where HUF_selectDecoder picks X2)
//   FSE headers          zstd/lib/common/entropy_common.c (FSE_readNCount, HUF_readStats),
//                        zstd/lib/common/fse_decompress.c (weights: two interleaved states)
// One wave per frame.  Entropy decoding is inherently sequential, so it runs as wave-uniform
// scalar code (every lane holds the same state; tables in LDS read at uniform addresses); the
// backward bitstreams are read through 512-byte register windows (v_readlane, no memory round
// trip per refill).  Literals are decoded into the tail of the chunk's own output region (the
// frame content size is known), and the sequences are executed with the LZ4 decoder's group
// emitter: up to 64 sequences per group, one output byte per lane per pass, through the LDS
// output window.
// Scope: frames as lzbench writes them (content size present, no dictionary), with or without the
// XXH64 content checksum (verified);
// others return kErrUnsupported.  Valid frames decode to the reference's bytes; corrupt frames
// are rejected without faulting, with the reference's accept / reject verdict (tests/test_gpu_zstd.py).
namespace zstdd {

constexpr int kZW = 2048;               // LDS output window (zstd offsets are mostly far anyway)
typedef owin::SinkT<kZW> ZSink;
constexpr int kErrCorrupt = -1, kErrUnsupported = -2, kErrChecksum = -1;

// XXH64 (seed 0) of out[0, len) -- /root/reference/zstd/lib/common/xxhash.h XXH64_endian_align --
// by the whole wave: lane j loads 32-byte stripe j of each 2 KiB batch (L1-bypassing: the bytes
// were just stored by this wave), the four accumulators take the stripes in order (wave-uniform)
__device__ __forceinline__ uint64_t xxh_rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xxh64_round(uint64_t acc, uint64_t in) {
    return xxh_rotl64(acc + in * 0xC2B2AE3D27D4EB4FULL, 31) * 0x9E3779B185EBCA87ULL;
}
__device__ uint64_t xxh64_wave(const Bytes& b, int len, int lane) {
    constexpr uint64_t P1 = 0x9E3779B185EBCA87ULL, P2 = 0xC2B2AE3D27D4EB4FULL, P3 = 0x165667B19E3779F9ULL,
                       P4 = 0x85EBCA77C2B2AE63ULL, P5 = 0x27D4EB2F165667C5ULL;
    auto rd32 = [&](int q) -> uint32_t {
        return b.b_sc1(q) | (b.b_sc1(q + 1) << 8) | (b.b_sc1(q + 2) << 16) | (b.b_sc1(q + 3) << 24);
    };
    uint64_t h;
    int p = 0;
    if (len >= 32) {
        uint64_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0ull - P1;
        const int ns = len / 32;
        for (int s0 = 0; s0 < ns; s0 += 64) {
            const int q = (s0 + lane) * 32;
            const bool in = s0 + lane < ns;
            uint32_t w[8];
#pragma unroll
            for (int k = 0; k < 8; k++) w[k] = in ? rd32(q + 4 * k) : 0u;
            const int m = min(64, ns - s0);
            for (int j = 0; j < m; j++) {
                v1 = xxh64_round(v1, (uint64_t)rdlane(w[1], j) << 32 | rdlane(w[0], j));
                v2 = xxh64_round(v2, (uint64_t)rdlane(w[3], j) << 32 | rdlane(w[2], j));
                v3 = xxh64_round(v3, (uint64_t)rdlane(w[5], j) << 32 | rdlane(w[4], j));
                v4 = xxh64_round(v4, (uint64_t)rdlane(w[7], j) << 32 | rdlane(w[6], j));
            }
        }
        p = ns * 32;
        h = xxh_rotl64(v1, 1) + xxh_rotl64(v2, 7) + xxh_rotl64(v3, 12) + xxh_rotl64(v4, 18);
        h = (h ^ xxh64_round(0, v1)) * P1 + P4;
        h = (h ^ xxh64_round(0, v2)) * P1 + P4;
        h = (h ^ xxh64_round(0, v3)) * P1 + P4;
        h = (h ^ xxh64_round(0, v4)) * P1 + P4;
    } else {
        h = P5;
    }
    h += (uint64_t)len;
    for (; p + 8 <= len; p += 8) {
        const uint64_t k = (uint64_t)uni(rd32(p + 4)) << 32 | uni(rd32(p));
        h = xxh_rotl64(h ^ xxh64_round(0, k), 27) * P1 + P4;
    }
    if (p + 4 <= len) {
        h = xxh_rotl64(h ^ ((uint64_t)uni(rd32(p)) * P1), 23) * P2 + P3;
        p += 4;
    }
    for (; p < len; p++) h = xxh_rotl64(h ^ ((uint64_t)uni(b.b_sc1(p)) * P5), 11) * P1;
    h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32;
    return h;
}
#ifndef LZH_ZSTD_DEBUG
#define LZH_ZSTD_DEBUG 0
#endif
// corrupt: -1, or (debug builds) -(10000 + source line) to locate the failing check
#define ZC (LZH_ZSTD_DEBUG ? -(10000 + __LINE__) : kErrCorrupt)
// phase clocks (debug builds with -DLZH_ZSTD_STATS=1; the launcher prints them)
#ifndef LZH_ZSTD_STATS
#define LZH_ZSTD_STATS 0
#endif
constexpr int kZClk = 8;
#define ZCLK(F, i) do { if (LZH_ZSTD_STATS) { const uint64_t t_ = __builtin_amdgcn_s_memtime(); (F).clk[i] += t_ - (F).clk_last; (F).clk_last = t_; } } while (0)
constexpr int kBlockMax = 128 * 1024;
constexpr int kHufLogMax = 12;          // HUF_TABLELOG_MAX (huf.h:119): the decoder accepts 12

// literal-length / match-length codes: baseline and extra bits (RFC 8878 3.1.1.3.2.1.1;
// common/zstd_internal.h LL_bits / ML_bits) and the predefined distributions (3.1.1.3.2.2;
// LL/ML/OF_defaultNorm)
__constant__ uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10,   11,   12,   13,    14,    15,    16,   18,
                                     20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14,  15,  16,  17,  18,   19,   20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32,  33,  34,  35,  37,   39,   41,
                                     43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ int8_t kLLNorm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int8_t kMLNorm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1,  1,  1,  1,  1,  1,  1,  1,  1,  1,  1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int8_t kOFNorm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

// FSE decoding-table cell, 32 bits: next-state base (9) | nbBits << 9 (4) | extra bits << 13 (5)
// | symbol << 18 (6).  For LL/ML the symbol is the length code (its baseline comes from a constant
// table off the state chain), for OF the offset code (= its extra-bit count).
typedef uint32_t Cell;
__device__ __forceinline__ uint32_t c_next(Cell c) { return c & 511u; }
__device__ __forceinline__ int c_nb(Cell c) { return (int)((c >> 9) & 15u); }
__device__ __forceinline__ int c_add(Cell c) { return (int)((c >> 13) & 31u); }
__device__ __forceinline__ uint32_t c_sym(Cell c) { return c >> 18; }

// per-wave LDS
struct Lds {
    uint16_t huf[1 << kHufLogMax];      // Huffman decoding table: symbol | nbBits << 8
    Cell ll[512], ml[512], of[256];     // sequence FSE tables (ZSTD_seqSymbol's fields, packed)
    Cell wt[64];                       // FSE table of the Huffman weights (accuracy <= 6)
    uint8_t weights[256];
    int16_t norm[256];
    uint16_t next[256];
    // (the split decoder's header kernel allocates the fields above only)
    uint32_t base[36 + 53];             // literal-length / match-length baselines (kLLBase, kMLBase)
    uint8_t win[kZW + 3 * LZH_WAVE];     // output window | start marks + scratch (groups::emit_group)
};
constexpr size_t kLdsHdr = offsetof(Lds, base);

__device__ __forceinline__ uint32_t lds_u32(const LDSA uint32_t* p) { return uni(*(volatile const LDSA uint32_t*)p); }
__device__ __forceinline__ uint32_t lds_u16(const LDSA uint16_t* p) { return uni(*(volatile const LDSA uint16_t*)p); }
__device__ __forceinline__ uint32_t lds_u8(const LDSA uint8_t* p) { return uni(*(volatile const LDSA uint8_t*)p); }
__device__ __forceinline__ Cell lds_cell(const LDSA Cell* p) { return uni(*(volatile const LDSA uint32_t*)p); }
__device__ __forceinline__ int hb32(uint32_t v) { return 31 - __builtin_clz(v); }   // v > 0

// uniform little-endian reads from a forward register window (Win) over the frame
__device__ __forceinline__ uint32_t fbyte(ZWin& w, int pos, int lane) { w.ensure(pos, lane); return uni(w.byte(pos)); }
__device__ __forceinline__ uint32_t fword(ZWin& w, int pos, int lane) {   // bytes pos..pos+3
    w.ensure(pos, lane);
    const int x = pos + w.sh, d = (x - w.wb) >> 2;
    const uint32_t a = d < 64 ? rdlane(w.w0, d) : rdlane(w.w1, d - 64);
    const uint32_t b = d + 1 < 64 ? rdlane(w.w0, d + 1) : rdlane(w.w1, d + 1 - 64);
    return uni(__builtin_amdgcn_alignbyte(b, a, (uint32_t)x & 3u));
}

// Backward bitstream (RFC 8878 4.1 / bitstream.h BIT_DStream), wave-uniform.  Positions are
// bit indices in the descriptor's byte space: the stream is bits [lo, P) still unread, the next
// n-bit field is bits [P - n, P) (most significant first).  c holds the 64 bits from the
// dword-aligned bit D8 (P - D8 in [32, 63] after a reload, so any field of <= 32 bits is in
// c); source dwords come from a 512-byte register window (v_readlane) that slides down.
struct BackBits {
    rsrc_t r;
    int wb;              // descriptor offset of the window start (multiple of 4)
    uint32_t w0, w1;     // window dwords [wb, wb + 256), [wb + 256, wb + 512)
    int lo, P, D8;
    uint64_t c;

    __device__ __forceinline__ uint32_t dw(int D) const {
        const int d = (D - wb) >> 2;
        return rdlane(d < 64 ? w0 : w1, d & 63);
    }
    __device__ __forceinline__ void cover(int D0, int D1, int lane) {   // bytes [D0, D1), D1 - D0 <= 256
        if (D0 >= wb && D1 <= wb + 512) return;
        if (D0 >= wb - 256 && D1 <= wb + 256) {
            w1 = w0;
            wb -= 256;
            w0 = ld_b32(r, wb + 4 * lane);
            return;
        }
        wb = D1 - 512;
        w0 = ld_b32(r, wb + 4 * lane);
        w1 = ld_b32(r, wb + 256 + 4 * lane);
    }
    __device__ __forceinline__ void reload(int lane) {
        D8 = ((P - 32) >> 5) << 5;
        const int D = D8 >> 3;
        cover(D, D + 8, lane);
        c = ((uint64_t)dw(D + 4) << 32) | dw(D);
    }
    // stream = descriptor bytes [start, start + size) (start including the descriptor shift);
    // false if empty or the end mark is missing
    __device__ __forceinline__ bool init(const Bytes& src, int start, int size, int lane) {
        r = src.r;
        const int s0 = start + src.sh;
        wb = ((s0 + size + 3) & ~3) - 512;
        w0 = ld_b32(r, wb + 4 * lane);
        w1 = ld_b32(r, wb + 256 + 4 * lane);
        lo = 8 * s0;
        if (size <= 0) return false;
        const int X = s0 + size - 1;
        const uint32_t last = (dw(X & ~3) >> (8 * (X & 3))) & 0xffu;
        if (last == 0) return false;
        P = 8 * X + hb32(last);
        reload(lane);
        return true;
    }
    __device__ __forceinline__ int left() const { return P - lo; }
    // next n bits (0 <= n <= 32), consumed; bits below the stream start read as garbage
    // (callers reject a stream that overruns)
    __device__ __forceinline__ uint32_t get(int n, int lane) {
        if (P - n < D8) reload(lane);
        const uint32_t v = (uint32_t)((c >> (P - n - D8)) & ((1ull << n) - 1ull));
        P -= n;
        return v;
    }
    // next n bits (1 <= n <= 32) without consuming them, zero-padded below the stream start
    __device__ __forceinline__ uint32_t peek(int n, int lane) {
        if (P - n < D8) reload(lane);
        uint32_t v = (uint32_t)((c >> (P - n - D8)) & ((1ull << n) - 1ull));
        if (P - n < lo) v &= (uint32_t)(~0ull << (lo - (P - n)));
        return v;
    }
    __device__ __forceinline__ void skip(int n) { P -= n; }
};

// value in a VGPR as far as the compiler knows (keeps wave-uniform chains out of the SGPR budget)
__device__ __forceinline__ int vgpr(int x) {
    int y;
    asm volatile("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
    return y;
}

// The sequences' backward bit stream with its state in vector registers (BackBits' container
// semantics): every read takes n <= 32 bits after making sure P - n >= D8, so a refill always
// moves the 64-bit container down by exactly one dword; the next eight dwords below are kept
// prefetched (bank a in use, bank b in flight).
struct SeqBits {
    rsrc_t r;
    int P, D8, lo, na, nxt;
    uint64_t c;
    uint32_t a0, a1, a2, a3, b0, b1, b2, b3;
    __device__ __forceinline__ bool init(const Bytes& src, int start, int size) {
        r = src.r;
        const int x0 = vgpr(start + src.sh);
        if (size <= 0) return false;
        const int X = x0 + size - 1;
        const uint32_t last = ld_u8(r, X);
        if (last == 0) return false;
        lo = 8 * x0;
        P = 8 * X + hb32(last);
        D8 = ((P - 32) >> 5) << 5;
        const int D = D8 >> 3;
        c = ((uint64_t)ld_b32(r, D + 4) << 32) | ld_b32(r, D);
        a0 = ld_b32(r, D - 4); a1 = ld_b32(r, D - 8); a2 = ld_b32(r, D - 12); a3 = ld_b32(r, D - 16);
        b0 = ld_b32(r, D - 20); b1 = ld_b32(r, D - 24); b2 = ld_b32(r, D - 28); b3 = ld_b32(r, D - 32);
        na = 4;
        nxt = D - 36;
        return true;
    }
    __device__ __forceinline__ int left() const { return P - lo; }
    __device__ __forceinline__ uint32_t get(int n) {
        if (P - n < D8) {
            c = (c << 32) | a0;
            a0 = a1; a1 = a2; a2 = a3;
            D8 -= 32;
            if (--na == 0) {
                a0 = b0; a1 = b1; a2 = b2; a3 = b3;
                b0 = ld_b32(r, nxt); b1 = ld_b32(r, nxt - 4); b2 = ld_b32(r, nxt - 8); b3 = ld_b32(r, nxt - 12);
                nxt -= 16;
                na = 4;
            }
        }
        const uint32_t v = (uint32_t)((c >> (P - n - D8)) & ((1ull << n) - 1ull));
        P -= n;
        return v;
    }
};

// FSE_readNCount (entropy_common.c:70-215) over the frame from byte pos: normalized counts
// into L.norm[0..maxSym], returns the header size in bytes (<= 0: corrupt); *al = accuracy log
__device__ __forceinline__ int read_ncount(ZWin& fw, int pos, int end, int maxSym, int maxLog, LDSA Lds& L, int& al, int& nsym,
                           int lane) {
    for (int i = lane; i < 256; i += LZH_WAVE) L.norm[i] = 0;
    int bit = 0;                                      // bits consumed from pos
    auto peek32 = [&](void) -> uint32_t {
        const int p = pos + (bit >> 3);
        const uint64_t v = ((uint64_t)fword(fw, p + 4, lane) << 32) | fword(fw, p, lane);
        return (uint32_t)(v >> (bit & 7));
    };
    uint32_t bs = peek32();
    int nb = (int)(bs & 15u) + 5;
    if (nb > maxLog) return ZC;
    al = nb;
    bit = 4;
    int remaining = (1 << nb) + 1, threshold = 1 << nb;
    nb++;
    int sym = 0;
    bool prev0 = false;
    for (int guard = 0; guard < 512; guard++) {
        if (prev0) {                                  // 2-bit repeat flags: 3 = three more zeros, go on
            for (int g2 = 0; g2 < 256; g2++) {
                const uint32_t r2 = peek32() & 3u;
                bit += 2;
                sym += (int)r2;
                if (r2 != 3) break;
            }
            if (sym > maxSym) return ZC;
        }
        bs = peek32();
        const int mx = (2 * threshold - 1) - remaining;
        int count;
        if ((int)(bs & (uint32_t)(threshold - 1)) < mx) {
            count = (int)(bs & (uint32_t)(threshold - 1));
            bit += nb - 1;
        } else {
            count = (int)(bs & (uint32_t)(2 * threshold - 1));
            if (count >= threshold) count -= mx;
            bit += nb;
        }
        count--;
        remaining -= count < 0 ? -count : count;
        if (sym > maxSym) return ZC;
        if (lane == 0) L.norm[sym] = (int16_t)count;
        sym++;
        prev0 = count == 0;
        if (remaining < threshold) {
            if (remaining <= 1) break;
            nb = hb32((uint32_t)remaining) + 1;
            threshold = 1 << (nb - 1);
        }
        if (sym > maxSym) break;
    }
    wave_lds_fence();
    if (remaining != 1 || bit > 8 * (end - pos)) return ZC;
    nsym = sym;
    return (bit + 7) >> 3;
}

// FSE_buildDTable (fse_decompress.c:72-160; ZSTD_buildFSETable for the sequence tables):
// symbols spread over the table, then each cell's next-state base and bit count.  Cells are
// (symbol, next-state base | nbBits << 16).
__device__ __forceinline__ void build_fse(LDSA Cell* T, int al, int nsym, LDSA Lds& L, int lane) {
    const int size = 1 << al, mask = size - 1;
    int high = size - 1;
    for (int s = 0; s < nsym; s++) {                  // low-probability symbols at the top
        const int n = (int16_t)lds_u16((const LDSA uint16_t*)&L.norm[s]);
        if (n == -1) {
            if (lane == 0) T[high] = (uint32_t)s << 18;
            high--;
        }
        if (lane == 0) L.next[s] = (uint16_t)(n == -1 ? 1 : n);
    }
    wave_lds_fence();
    const int step = (size >> 1) + (size >> 3) + 3;
    int p = 0;
    for (int s = 0; s < nsym; s++) {
        const int n = (int16_t)lds_u16((const LDSA uint16_t*)&L.norm[s]);
        for (int i = 0; i < n; i++) {
            if (lane == 0) T[p] = (uint32_t)s << 18;
            p = (p + step) & mask;
            while (p > high) p = (p + step) & mask;
        }
    }
    wave_lds_fence();
    for (int u = 0; u < size; u++) {
        const uint32_t s = uni(((volatile const LDSA uint32_t*)T)[u]) >> 18;
        const uint32_t nx = lds_u16(&L.next[s]);
        if (lane == 0) L.next[s] = (uint16_t)(nx + 1);
        const int nb = al - hb32(nx);
        const uint32_t base = (nx << nb) - (uint32_t)size;
        if (lane == 0) T[u] = (s << 18) | ((uint32_t)nb << 9) | base;
        wave_lds_fence();
    }
}

// FSE_buildDTable for the sequence tables (nsym <= 53, size <= 512), lane-parallel, the same cells as
// build_fse: (1) per symbol (lanes): the low-probability symbols' top cells and the running sum C of
// the other counts; (2) per spread step i (lanes, 64 at a time): position (i * step) & mask, kept when
// <= high, its rank among the kept ones gives the symbol (the last s with C[s] <= rank: a binary
// search); (3) per position u ascending (lanes, 64 at a time): the symbol's next-state counter value
// at u -- its initial count plus the same-symbol cells before u -- with the counters in one VGPR
// (lane s holds symbol s's) and the cells of a 64-position batch taken one distinct symbol at a time.
__device__ __forceinline__ void build_fse_par(LDSA Cell* T, int al, int nsym, LDSA Lds& L, int lane) {
    const int size = 1 << al, mask = size - 1;
    const int step = (size >> 1) + (size >> 3) + 3;
    const uint64_t below = (1ull << lane) - 1ull;
    // (1) symbols: lane s (nsym <= 64)
    const int n = lane < nsym ? (int)L.norm[lane] : 0;
    const bool lowp = n == -1;
    const uint64_t lm = ballot(lowp);
    const int nlow = __builtin_popcountll(lm);
    const int high = size - 1 - nlow;
    if (lowp) T[size - 1 - __builtin_popcountll(lm & below)] = (uint32_t)lane << 18;
    int C = n > 0 ? n : 0;                            // exclusive prefix sum of the positive counts
    {
        int x = C;
#pragma unroll
        for (int k = 1; k < 64; k <<= 1) {
            const int y = __shfl_up(x, k);
            if (lane >= k) x += y;
        }
        C = x - C;
    }
    L.next[lane < 256 ? lane : 0] = lane < nsym ? (uint16_t)C : (uint16_t)0xffffu;
    wave_lds_fence();
    // (2) the spread
    int kept = 0;
    for (int c = 0; c < size; c += LZH_WAVE) {
        const int i = c + lane;
        const int pos = (int)(((uint32_t)i * (uint32_t)step) & (uint32_t)mask);
        const bool valid = i < size && pos <= high;
        const uint64_t vm = ballot(valid);
        const int rank = kept + __builtin_popcountll(vm & below);
        kept += __builtin_popcountll(vm);
        // the last symbol s < nsym with C[s] <= rank
        int lo = 0, hi = nsym - 1;
        while (ballot(valid && lo < hi)) {
            const int mid = (lo + hi + 1) >> 1;
            const bool le = (int)L.next[mid] <= rank;
            if (valid && lo < hi) { lo = le ? mid : lo; hi = le ? hi : mid - 1; }
        }
        if (valid) T[pos] = (uint32_t)lo << 18;
    }
    wave_lds_fence();
    // (3) next states, positions ascending
    int cnt = lowp ? 1 : n;                           // lane s: symbol s's counter
    for (int c = 0; c < size; c += LZH_WAVE) {
        const int u = c + lane;
        const bool on = u < size;
        const uint32_t sym = on ? (T[u] >> 18) : 0xffu;
        int nx = 0;
        for (uint64_t rem = ballot(on); rem;) {
            const int s0 = (int)rdlane(sym, __builtin_ctzll(rem));
            const uint64_t m = ballot(on && sym == (uint32_t)s0) & rem;
            const int base = rdlanei(cnt, s0);
            if (lane_on(m)) nx = base + __builtin_popcountll(m & below);
            if (lane == s0) cnt += __builtin_popcountll(m);
            rem &= ~m;
        }
        if (on) {
            const int nb = al - hb32((uint32_t)nx);
            const uint32_t base = ((uint32_t)nx << nb) - (uint32_t)size;
            T[u] = (sym << 18) | ((uint32_t)nb << 9) | base;
        }
    }
    wave_lds_fence();
}

// sequence-table cells: symbol -> baseline value and extra-bit count (RFC 8878 3.1.1.3.2.1.1)
__device__ __forceinline__ void seq_cells(LDSA Cell* T, int size, int which, int lane) {
    for (int u = lane; u < size; u += LZH_WAVE) {
        const uint32_t c = T[u], s = c >> 18;
        const uint32_t add = which == 0 ? kLLBits[s] : (which == 2 ? kMLBits[s] : s);
        T[u] = c | (add << 13);
    }
    wave_lds_fence();
}

// sequence table for one of LL / OF / ML (ZSTD_buildSeqTable, zstd_decompress_block.c:~560):
// mode 0 predefined, 1 RLE, 2 FSE-compressed, 3 repeat.  Returns bytes consumed, < 0 corrupt.
__device__ __forceinline__ int seq_table(ZWin& fw, int pos, int end, int mode, int which, LDSA Cell* T, int& al, bool& valid,
                         LDSA Lds& L, int lane) {
    const int maxSym = which == 0 ? 35 : (which == 1 ? 31 : 52);
    const int maxLog = which == 1 ? 8 : 9;
    if (mode == 0) {
        const int n = which == 0 ? 36 : (which == 1 ? 29 : 53);
        for (int s = lane; s < n; s += LZH_WAVE)
            L.norm[s] = which == 0 ? kLLNorm[s] : (which == 1 ? kOFNorm[s] : kMLNorm[s]);
        wave_lds_fence();
        al = which == 1 ? 5 : 6;
        build_fse_par(T, al, n, L, lane);
        seq_cells(T, 1 << al, which, lane);
        valid = true;
        return 0;
    }
    if (mode == 1) {
        if (pos >= end) return ZC;
        const int s = (int)fbyte(fw, pos, lane);
        if (s > maxSym) return ZC;
        if (lane == 0) T[0] = (uint32_t)s << 18;
        wave_lds_fence();
        seq_cells(T, 1, which, lane);
        al = 0;
        valid = true;
        return 1;
    }
    if (mode == 2) {
        int nsym = 0;
        const int h = read_ncount(fw, pos, end, maxSym, maxLog, L, al, nsym, lane);
        if (h <= 0) return h < 0 ? h : ZC;
        if (pos + h > end) return ZC;
        build_fse_par(T, al, nsym, L, lane);
        seq_cells(T, 1 << al, which, lane);
        valid = true;
        return h;
    }
    return valid ? 0 : -1;                             // repeat: the previous block's table
}

// Huffman tree description (HUF_readStats, entropy_common.c:271-334; HUF_readDTableX1,
// huf_decompress.c:342-470) at pos.  Returns bytes consumed (< 0 corrupt), *tl = table log.
__device__ __forceinline__ int read_huf(ZWin& fw, const Bytes& src, int pos, int end, LDSA Lds& L, int& tl, int lane) {
    if (pos >= end) return ZC;
    const int hb = (int)fbyte(fw, pos, lane);
    int n, used;
    if (hb >= 128) {                                   // direct 4-bit weights
        n = hb - 127;
        used = 1 + (n + 1) / 2;
        if (pos + used > end) return ZC;
        for (int i = 0; i < n; i++) {
            const uint32_t b = fbyte(fw, pos + 1 + i / 2, lane);
            if (lane == 0) L.weights[i] = (uint8_t)((i & 1) ? (b & 15u) : (b >> 4));
        }
    } else {                                           // FSE-compressed weights, accuracy <= 6
        used = 1 + hb;
        if (pos + used > end || hb == 0) return ZC;
        int al = 0, nsym = 0;
        const int h = read_ncount(fw, pos + 1, pos + 1 + hb, 255, 6, L, al, nsym, lane);
        if (h < 0) return h;
        if (h == 0 || h >= hb) return ZC;
        build_fse(L.wt, al, nsym, L, lane);
        BackBits bb;
        if (!bb.init(src, pos + 1 + h, hb - h, lane)) return ZC;
        // two interleaved states (fse_decompress.c:199-250): after each symbol's state
        // update, an exhausted stream ends with one more symbol from the other state
        uint32_t s1 = bb.get(al, lane), s2 = bb.get(al, lane);
        n = 0;
        for (int k = 0;; k ^= 1) {
            if (n > 253) return ZC;
            const Cell e = lds_cell(&L.wt[k ? s2 : s1]);
            if (lane == 0) L.weights[n] = (uint8_t)c_sym(e);
            n++;
            const uint32_t ns = c_next(e) + bb.get(c_nb(e), lane);
            if (k) s2 = ns; else s1 = ns;
            if (bb.left() < 0) {
                const Cell e2 = lds_cell(&L.wt[k ? s1 : s2]);
                if (lane == 0) L.weights[n] = (uint8_t)c_sym(e2);
                n++;
                break;
            }
        }
    }
    wave_lds_fence();
    // weights -> table log, the implied last weight (HUF_readStats: a clean power of 2 completes
    // the total), at least two and an even number of weight-1 symbols
    uint32_t total = 0;
    int c1 = 0;
    for (int i = 0; i < n; i++) {
        const int w = (int)lds_u8(&L.weights[i]);
        if (w > 12) return ZC;
        c1 += w == 1;
        total += (1u << w) >> 1;
    }
    if (total == 0) return ZC;
    tl = hb32(total) + 1;
    if (tl > 12) return ZC;
    if (tl > kHufLogMax) return kErrUnsupported;
    const uint32_t rest = (1u << tl) - total;
    if (rest & (rest - 1)) return ZC;
    const int lw = hb32(rest) + 1;
    if (lane == 0) L.weights[n] = (uint8_t)lw;
    c1 += lw == 1;
    n++;
    if (c1 < 2 || (c1 & 1)) return ZC;
    wave_lds_fence();
    // table (HUF_readDTableX1): weight 1 first, symbols in order within a weight, 2^(w-1) cells
    // each; symbols of a weight found by ballot over the 4 x 64 weights held in registers
    uint32_t wv[4];
#pragma unroll
    for (int j = 0; j < 4; j++) wv[j] = lane + 64 * j < n ? (uint32_t)L.weights[lane + 64 * j] : 0u;
    int start = 0;
    for (int w = 1; w <= tl; w++) {
        const int len = 1 << (w - 1);
        const uint32_t cell = (uint32_t)(tl + 1 - w) << 8;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            for (uint64_t m = ballot(wv[j] == (uint32_t)w); m; m &= m - 1) {
                const uint32_t s = (uint32_t)(__builtin_ctzll(m) + 64 * j);
                for (int i = lane; i < len; i += LZH_WAVE) L.huf[start + i] = (uint16_t)(cell | s);
                start += len;
            }
        }
    }
    wave_lds_fence();
    return used;
}

// literals of one Huffman stream set into out[dst .. dst + rs): 1 or 4 streams (1X1 / 4X1,
// huf_decompress.c HUF_decompress1X1 / 4X1_usingDTable), one stream per lane.  Lane j holds
// stream j's backward bit container as in BackBits (64 bits c at bit offset D8, position P): a
// container refill always moves down by exactly one dword (P - tl < D8 happens only once P is
// within tl bits of D8), so the next dwords below are prefetched per lane, four at a time
// (bank a in use, bank b in flight); the symbol lookup is a per-lane LDS read and each step
// stores one byte per stream.  The streams' decoding chains run side by side in the lanes.
__device__ __forceinline__ int huf_streams(const Bytes& src, int pos, int csize, int nstreams, const Bytes& out, int dst, int rs,
                            int tl, LDSA Lds& L, int lane) {
    int seg = rs, last = rs, s0 = pos, sz = csize;   // this lane's stream: [s0, s0 + sz), seg (or last) symbols
    if (nstreams == 4) {
        if (csize < 10) return ZC;
        ZWin fw;
        fw.bind(src, nullptr);
        fw.load(pos, lane);
        const int z1 = (int)(fword(fw, pos, lane) & 0xffffu), z2 = (int)(fword(fw, pos + 2, lane) & 0xffffu),
                  z3 = (int)(fword(fw, pos + 4, lane) & 0xffffu);
        const int z4 = csize - 6 - z1 - z2 - z3;
        if (z4 < 1) return ZC;
        seg = (rs + 3) / 4;
        last = rs - 3 * seg;
        if (last < 0) return ZC;
        if (z1 <= 0 || z2 <= 0 || z3 <= 0) return ZC;
        const int p1 = pos + 6;
        s0 = lane == 0 ? p1 : (lane == 1 ? p1 + z1 : (lane == 2 ? p1 + z1 + z2 : p1 + z1 + z2 + z3));
        sz = lane == 0 ? z1 : (lane == 1 ? z2 : (lane == 2 ? z3 : z4));
    } else if (csize <= 0) {
        return ZC;
    }
    const bool on = lane < nstreams;
    const int nsym = lane == 3 ? last : seg;           // symbols of this lane's stream
    const rsrc_t r = src.r;
    const int x0 = s0 + src.sh;
    const int X = x0 + sz - 1;                          // the stream's last byte holds the end mark
    const uint32_t lastb = on ? ld_u8(r, X) : 1u;
    if (ballot(on && lastb == 0)) return ZC;
    const int lo = 8 * x0;
    int P = 8 * X + hb32(lastb);
    int D8 = ((P - 32) >> 5) << 5;
    int D = D8 >> 3;                                    // (dword aligned; below 0 reads as 0)
    uint64_t c = on ? (((uint64_t)ld_b32(r, D + 4) << 32) | ld_b32(r, D)) : 0ull;
    uint32_t a0 = 0, a1 = 0, a2 = 0, a3 = 0, b0 = 0, b1 = 0, b2 = 0, b3 = 0;
    if (on) {
        a0 = ld_b32(r, D - 4); a1 = ld_b32(r, D - 8); a2 = ld_b32(r, D - 12); a3 = ld_b32(r, D - 16);
        b0 = ld_b32(r, D - 20); b1 = ld_b32(r, D - 24); b2 = ld_b32(r, D - 28); b3 = ld_b32(r, D - 32);
    }
    int na = 4, nxt = D - 36;                           // dwords left in bank a; next dword to fetch
    const uint32_t mask = (1u << tl) - 1u;
    for (int i = 0; i < seg; i++) {
        const bool act = on && i < nsym;
        if (act && P - tl < D8) {                       // container refill: one dword down
            c = (c << 32) | a0;
            a0 = a1; a1 = a2; a2 = a3;
            D8 -= 32;
            if (--na == 0) {                            // bank b becomes a, the next four are fetched
                a0 = b0; a1 = b1; a2 = b2; a3 = b3;
                b0 = ld_b32(r, nxt); b1 = ld_b32(r, nxt - 4); b2 = ld_b32(r, nxt - 8); b3 = ld_b32(r, nxt - 12);
                nxt -= 16;
                na = 4;
            }
        }
        const int sh = P - tl - D8;
        uint32_t v = (uint32_t)(c >> (sh & 63)) & mask;
        if (P - tl < lo) v &= (uint32_t)(~0ull << min(lo - (P - tl), 63));   // zero-padded below the start
        const uint32_t e = ((volatile const LDSA uint16_t*)L.huf)[act ? v : 0];
        if (act) {
            P -= (int)(e >> 8);
            out.st8(dst + lane * seg + i, e & 0xffu);
        }
    }
    return ballot(on && P != lo) ? 1 : 0;              // 1: some stream not exactly consumed
}

// HUF_selectDecoder (huf_decompress.c:1565-1615): 1 when the reference decodes a 4-stream literal
// section it has just read a tree for with the double-symbol decoder (X2)
__constant__ uint16_t kAlgoTime[16][4] = {
    {0, 0, 1, 1}, {0, 0, 1, 1}, {150, 216, 381, 119}, {170, 205, 514, 112}, {177, 199, 539, 110},
    {197, 194, 644, 107}, {221, 192, 735, 107}, {256, 189, 881, 106}, {359, 188, 1167, 109},
    {582, 187, 1570, 114}, {688, 187, 1712, 122}, {825, 186, 1965, 136}, {976, 185, 2131, 150},
    {1180, 186, 2070, 175}, {1377, 185, 1731, 202}, {1412, 185, 1695, 202}};
__device__ __forceinline__ bool huf_select_x2(int dstSize, int cSrcSize) {
    const int Q = cSrcSize >= dstSize ? 15 : (int)((uint32_t)cSrcSize * 16u / (uint32_t)dstSize);
    const uint32_t D256 = (uint32_t)dstSize >> 8;
    const uint32_t t0 = kAlgoTime[Q][0] + kAlgoTime[Q][1] * D256;
    uint32_t t1 = kAlgoTime[Q][2] + kAlgoTime[Q][3] * D256;
    t1 += t1 >> 5;
    return t1 < t0;
}

// The double-symbol decoder's verdict (HUF_decompress1X2 / 4X2_usingDTable_internal_body,
// huf_decompress.c:1176-1363), run when the single-symbol walk of huf_streams did not consume some
// stream exactly and the reference table is X2.  Both decoders emit the same symbols wherever the
// bits are read inside the stream (an X2 cell of targetLog = max(11, tl) bits holds the next code
// and, when both fit, the code after it: HUF_fillDTableX2), and a stream X1 accepts X2 accepts
// with the same bytes.  X2 differs on corrupt streams in three ways, restated here per lane (one
// stream per lane, lookups in lock step):
//  * the last symbol of a stream (HUF_decodeLastSymbolX2, :1148-1163): a two-symbol cell skips
//    both codes and clamps an overrun to the stream start, so the stream ends exactly consumed
//    whenever it had bits left; with none left the cell comes from the top bits of the 64-bit
//    container loaded at the stream start (bitsConsumed == 64: the shift wraps to 0);
//  * the 4-stream loop (:1294-1342) decodes 4 cells per stream per round, 1 or 2 symbols each,
//    until some stream's reload pointer is within 8 bytes of its start or stream 4 is within 7
//    bytes of its end; a stream 1..3 that wrote past its segment by then is corrupt (:1345-1347).
//    After a round's reload the pointer is ceil(r / 8) - 8 bytes above the stream start
//    (BIT_reloadDStreamFast, r = bits left), before the first one srcSize - 8 (or 0 below 8 bytes);
//  * anything consumed below the stream start is never recovered (bitsConsumed > 64), except by
//    the last-symbol clamp above.
// Symbols are written in place of the X1 walk's; returns 0 (accepted) or ZC.
__device__ __attribute__((noinline)) int huf_streams_x2(const Bytes& src, int pos, int csize, int nstreams, const Bytes& out,
                                                         int dst, int rs, int tl, LDSA Lds& L, int lane) {
    const rsrc_t r = src.r;
    int seg = rs, last = rs, s0 = pos, sz = csize;
    if (nstreams == 4) {                               // (geometry validated by huf_streams)
        const int b = pos + src.sh;
        const int z1 = (int)(ld_u8(r, b) | ld_u8(r, b + 1) << 8), z2 = (int)(ld_u8(r, b + 2) | ld_u8(r, b + 3) << 8),
                  z3 = (int)(ld_u8(r, b + 4) | ld_u8(r, b + 5) << 8);
        seg = (rs + 3) / 4;
        last = rs - 3 * seg;
        const int p1 = pos + 6;
        s0 = lane == 0 ? p1 : (lane == 1 ? p1 + z1 : (lane == 2 ? p1 + z1 + z2 : p1 + z1 + z2 + z3));
        sz = lane == 0 ? z1 : (lane == 1 ? z2 : (lane == 2 ? z3 : csize - 6 - z1 - z2 - z3));
    }
    const bool on = lane < nstreams;
    const int nsym = lane == 3 ? last : seg;
    const int x0 = s0 + src.sh, lo = 8 * x0, X = x0 + sz - 1;
    const uint32_t lastb = on ? ld_u8(r, X) : 1u;
    int P = 8 * X + hb32(lastb | 1u);
    const int T = tl <= 11 ? 11 : 12;                  // HUF_readDTableX2: maxTableLog, :1081
    const uint32_t tmask = (1u << T) - 1u;
    const uint32_t b6 = on && sz >= 7 ? ld_u8(r, x0 + 6) : 0u, b7 = on && sz >= 8 ? ld_u8(r, x0 + 7) : 0u;
    const uint32_t top = ((b7 << 8) | b6) >> (16 - T);   // BIT_initDStream's container, top T bits
    int q = sz >= 8 ? sz - 8 : 0;                      // reload pointer - start, bytes
    bool joint = nstreams == 4 && last >= 8;           // (oend - op4 >= 8 and op4 < olimit)
    int op = 0;
    for (int t = 0;; t++) {
        if (joint && t > 0 && (t & 3) == 0) {          // end of a round: the four reloads, the loop test
            const bool cont = q >= 8 && !(lane == 3 && op >= last - 7);
            if (ballot(on && !cont)) {
                joint = false;
                if (ballot(on && lane < 3 && op > seg)) return ZC;
            } else {
                q = ((P - lo + 7) >> 3) - 8;
            }
        }
        const bool act = on && (joint || op < nsym);
        if (!ballot(act)) break;
        if (!act) continue;
        uint32_t v;
        if (P == lo) {
            v = top;
        } else {
            const int qb = (P - T) >> 3, sh = (P - T) & 7;
            const uint32_t w = ld_u8(r, qb) | ld_u8(r, qb + 1) << 8 | ld_u8(r, qb + 2) << 16;
            v = (w >> sh) & tmask;
            if (P - T < lo) v &= (uint32_t)(~0ull << min(lo - (P - T), 32));   // zero-padded below the start
        }
        const uint32_t e1 = ((volatile const LDSA uint16_t*)L.huf)[v >> (T - tl)];
        const int n1 = (int)(e1 >> 8);
        const uint32_t e2 = ((volatile const LDSA uint16_t*)L.huf)[((v << n1) & tmask) >> (T - tl)];
        const int n2 = (int)(e2 >> 8);
        const bool dbl = n1 + n2 <= T;
        if (op < nsym) out.st8(dst + lane * seg + op, e1 & 0xffu);
        if (!joint && op == nsym - 1) {                // HUF_decodeLastSymbolX2
            if (!dbl) P -= n1;
            else if (P > lo) P = max(P - n1 - n2, lo);
            op++;
        } else {
            if (dbl && op + 1 < nsym) out.st8(dst + lane * seg + op + 1, e2 & 0xffu);
            P -= dbl ? n1 + n2 : n1;
            op += dbl ? 2 : 1;
        }
    }
    return ballot(on && P != lo) ? ZC : 0;
}

struct FrameState {
    int rep0, rep1, rep2;
    int llA, ofA, mlA;                  // accuracy logs of the current tables
    bool llV, ofV, mlV, hufV;           // tables valid for "repeat" / treeless modes
    bool hufX2;                         // the reference's table type (HUF_DTable tableType: 1 = X2)
    int hufTl;
    uint64_t clk[kZClk], clk_last;      // (LZH_ZSTD_STATS)
};

// one compressed block [bs, be) of the frame; output continues at op (returns new op, < 0 error)
__device__ __forceinline__ int decode_block(const Bytes& rin, const Bytes& lout, ZWin& fw, ZWin& lw, ZSink& O, LDSA Lds& L,
                            FrameState& F, int bs, int be, int op, int fcs, int lane) {
    // ---- literals section (ZSTD_decodeLiteralsBlock)
    const uint32_t b0 = fbyte(fw, bs, lane);
    const int ltype = (int)(b0 & 3u), sf = (int)((b0 >> 2) & 3u);
    int rs, lpos, seqpos;
    Bytes lsrc;                                       // where the literals are read from
    if (ltype <= 1) {
        int hsz;
        if ((sf & 1) == 0) { hsz = 1; rs = (int)(b0 >> 3); }
        else if (sf == 1) { hsz = 2; rs = (int)((b0 >> 4) + (fbyte(fw, bs + 1, lane) << 4)); }
        else { hsz = 3; rs = (int)((b0 >> 4) + (fbyte(fw, bs + 1, lane) << 4) + (fbyte(fw, bs + 2, lane) << 12)); }
        if (rs > kBlockMax) return ZC;
        if (ltype == 0) {
            if (bs + hsz + rs > be) return ZC;
            lsrc = rin;
            lpos = bs + hsz;
            seqpos = bs + hsz + rs;
        } else {
            if (bs + hsz + 1 > be || rs > fcs - op) return ZC;
            const uint32_t v = fbyte(fw, bs + hsz, lane);
            lsrc = lout;
            lpos = fcs - rs;
            for (int i = lane; i < rs; i += LZH_WAVE) O.out.st8(lpos + i, v);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            seqpos = bs + hsz + 1;
        }
    } else {
        const int hsz = sf <= 1 ? 3 : (sf == 2 ? 4 : 5);
        const int bits = sf <= 1 ? 10 : (sf == 2 ? 14 : 18);
        if (bs + hsz > be) return ZC;
        uint64_t h = 0;
        for (int i = 0; i < hsz; i++) h |= (uint64_t)fbyte(fw, bs + i, lane) << (8 * i);
        rs = (int)((h >> 4) & ((1u << bits) - 1));
        const int cs = (int)((h >> (4 + bits)) & ((1u << bits) - 1));
        if (rs > kBlockMax || bs + hsz + cs > be || rs > fcs - op) return ZC;
        int p = bs + hsz;
        if (ltype == 2) {
            int tl = 0;
            ZCLK(F, 0);
            const int u = read_huf(fw, rin, p, bs + hsz + cs, L, tl, lane);
            ZCLK(F, 1);
            if (u < 0) return u;
            F.hufV = true;
            F.hufTl = tl;
            // (ZSTD_decodeLiteralsBlock: a 1-stream tree is read as X1, a 4-stream one by HUF_selectDecoder)
            F.hufX2 = sf != 0 && huf_select_x2(rs, cs);
            p += u;
        } else if (!F.hufV) {
            return ZC;
        }
        lsrc = lout;
        lpos = fcs - rs;
        ZCLK(F, 0);
        if (rs == 0 && sf != 0 && ltype == 2) return ZC;   // HUF_decompress4X_hufOnly: dstSize 0
        int hr = huf_streams(rin, p, bs + hsz + cs - p, sf == 0 ? 1 : 4, O.out, lpos, rs, F.hufTl, L, lane);
        if (hr == 1)
            hr = F.hufX2 ? huf_streams_x2(rin, p, bs + hsz + cs - p, sf == 0 ? 1 : 4, O.out, lpos, rs, F.hufTl, L, lane) : ZC;
        ZCLK(F, 2);
        if (hr < 0) return hr;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // literal stores visible to the window loads
        seqpos = bs + hsz + cs;
    }
    lw.bind(lsrc, nullptr);
    lw.load(lpos, lane);

    // ---- sequences section header (ZSTD_decodeSeqHeaders)
    if (seqpos >= be) return ZC;
    int p = seqpos;
    int nseq = (int)fbyte(fw, p++, lane);
    if (nseq >= 128) {
        if (nseq == 255) {
            if (p + 2 > be) return ZC;
            nseq = (int)(fbyte(fw, p, lane) + (fbyte(fw, p + 1, lane) << 8)) + 0x7F00;
            p += 2;
        } else {
            if (p + 1 > be) return ZC;
            nseq = ((nseq - 128) << 8) + (int)fbyte(fw, p++, lane);
        }
    }
    int lp = 0;                                       // literals consumed
    if (nseq > 0) {
        if (p >= be) return ZC;
        const uint32_t modes = fbyte(fw, p++, lane);
        if (modes & 3u) return ZC;
        ZCLK(F, 0);
        int u = seq_table(fw, p, be, (int)(modes >> 6), 0, L.ll, F.llA, F.llV, L, lane);
        if (u < 0) return ZC;
        p += u;
        u = seq_table(fw, p, be, (int)((modes >> 4) & 3u), 1, L.of, F.ofA, F.ofV, L, lane);
        if (u < 0) return ZC;
        p += u;
        u = seq_table(fw, p, be, (int)((modes >> 2) & 3u), 2, L.ml, F.mlA, F.mlV, L, lane);
        if (u < 0) return ZC;
        p += u;
        // ---- sequences (ZSTD_decodeSequence), executed a group at a time.  The decoding chain
        // (bit reader, FSE states, repcodes, lengths, the group being filled) lives in vector
        // registers (every lane holds the same value: vgpr() hides the uniformity from the
        // compiler), so the frame's scalar state is not spilled to VGPR lanes and back around
        // every sequence; table lookups are LDS reads at one address per wave.
        ZCLK(F, 3);
        SeqBits sb;
        if (!sb.init(rin, p, be - p)) return ZC;
        uint32_t sLL = sb.get(F.llA), sOF = sb.get(F.ofA), sML = sb.get(F.mlA);
        int rep0 = vgpr(F.rep0), rep1 = vgpr(F.rep1), rep2 = vgpr(F.rep2);
        int k = vgpr(0), glit = vgpr(0), gout = vgpr(0);   // group: members, literal bytes, output bytes
        const int lrem0 = vgpr(rs - lp), opv = vgpr(op), fcsv = vgpr(fcs);
        uint32_t g_lit = 0, g_ml = 0, g_off = 0, g_ex = 0, g_lrel = 0;
        const volatile LDSA uint32_t* llT = (const volatile LDSA uint32_t*)L.ll;
        const volatile LDSA uint32_t* mlT = (const volatile LDSA uint32_t*)L.ml;
        const volatile LDSA uint32_t* ofT = (const volatile LDSA uint32_t*)L.of;
        int lpv = 0, opg = 0;                         // literals / output bytes of the groups emitted
        for (int i = 0; i < nseq; i++) {
            const Cell eL = llT[sLL], eO = ofT[sOF], eM = mlT[sML];
            const int ofc = (int)c_sym(eO);
            const int llc = (int)c_sym(eL), mlc = (int)c_sym(eM);
            const int ll0 = llc == 0;                 // (only literal-length code 0 has baseline 0)
            int off;
            if (ofc > 1) {
                off = (int)((1u << ofc) - 3u + sb.get(ofc));
                rep2 = rep1; rep1 = rep0; rep0 = off;
            } else if (ofc == 0) {
                off = ll0 ? rep1 : rep0;
                if (ll0) { rep1 = rep0; rep0 = off; }
            } else {
                const int idx = 1 + ll0 + (int)sb.get(1);   // 1..3
                int t = idx == 3 ? rep0 - 1 : (idx == 1 ? rep1 : rep2);
                t += t == 0;                          // (as the reference: offset 0 becomes 1)
                if (idx != 1) rep2 = rep1;
                rep1 = rep0;
                rep0 = off = t;
            }
            // match-length then literal-length extra bits (<= 16 each), one read of both
            const int am = c_add(eM), al = c_add(eL);
            const uint32_t xb = sb.get(am + al);
            const int ml = (int)L.base[36 + mlc] + (int)(xb >> al);
            const int ll = (int)L.base[llc] + (int)(xb & ((1u << al) - 1u));
            if (i + 1 < nseq) {                       // state updates LL, ML, OF: one read (<= 27 bits)
                const int nl = c_nb(eL), nm = c_nb(eM), no = c_nb(eO);
                const uint32_t sbits = sb.get(nl + nm + no);
                sLL = c_next(eL) + (sbits >> (nm + no));
                sML = c_next(eM) + ((sbits >> no) & ((1u << nm) - 1u));
                sOF = c_next(eO) + (sbits & ((1u << no) - 1u));
                if (sb.left() < 0) return ZC;
            } else {
                // the reference also updates the states after the last sequence and then accepts
                // an exhausted or overrun stream (ZSTD_decompressSequences_body: reload >= completed)
                const int extra = c_nb(eL) + c_nb(eM) + c_nb(eO);
                if (sb.left() > extra || sb.left() < 0) return ZC;
            }
            // validity (ZSTD_execSequence): literals available, offset within the output, room
            const int lrem = lrem0 - lpv - glit;      // literals not yet taken
            const int o0 = opv + opg + gout;          // output position of this sequence
            // (an offset code of 31 gives 2^31 - 3 + bits: compared unsigned, as the reference's size_t)
            if (ll > lrem || (uint32_t)off > (uint32_t)(o0 + ll) || (int64_t)o0 + ll + ml > (int64_t)(fcsv - (lrem - ll)))
                return ZC;
            const bool big = ll > 255 || ml > 4095;
            if (big || k == LZH_WAVE || glit + ll > 384) {
                // emit the pending group
                if (k > 0) {
                    const int kk = unii(k), gl = unii(glit), go = unii(gout), lpu = unii(lpv), opu = unii(op + opg);
                    const int ip = lpos + lp + lpu;
                    if (!lw.covers(ip, ip + gl + 16)) lw.load(ip, lane);
                    const uint64_t keep = kk == LZH_WAVE ? ~0ull : ((1ull << kk) - 1ull);
                    ZCLK(F, 4);
                    groups::emit_group(lw, O, (LDSA uint8_t*)L.win + kZW, ip, opu, go, keep, (int)g_ex,
                                       g_lit | (g_ml << 16), g_lrel, (int)g_off, lane);
                    ZCLK(F, 5);
                    opg += gout;
                    lpv += glit;
                    k = 0; glit = 0; gout = 0;
                }
                if (big) {                            // a long sequence on its own
                    const int bl = unii(ll), bm = unii(ml), bo = unii(off), lpu = unii(lpv), opu = unii(op + opg);
                    ZCLK(F, 4);
                    O.literals(lw, lsrc, lpos + lp + lpu, opu, bl, lane);
                    O.match(opu + bl, bo, bm, lane);
                    ZCLK(F, 6);
                    opg += ll + ml;
                    lpv += ll;
                    continue;
                }
            }
            g_lit = lane == k ? (uint32_t)ll : g_lit;
            g_ml = lane == k ? (uint32_t)ml : g_ml;
            g_off = lane == k ? (uint32_t)off : g_off;
            g_ex = lane == k ? (uint32_t)gout : g_ex;
            g_lrel = lane == k ? (uint32_t)glit : g_lrel;
            k++;
            glit += ll;
            gout += ll + ml;
        }
        if (unii(k) > 0) {
            const int kk = unii(k), gl = unii(glit), go = unii(gout), lpu = unii(lpv), opu = unii(op + opg);
            const int ip = lpos + lp + lpu;
            if (!lw.covers(ip, ip + gl + 16)) lw.load(ip, lane);
            const uint64_t keep = kk == LZH_WAVE ? ~0ull : ((1ull << kk) - 1ull);
            ZCLK(F, 4);
            groups::emit_group(lw, O, (LDSA uint8_t*)L.win + kZW, ip, opu, go, keep, (int)g_ex, g_lit | (g_ml << 16),
                               g_lrel, (int)g_off, lane);
            ZCLK(F, 5);
            opg += gout;
            lpv += glit;
        }
        op += unii(opg);
        lp += unii(lpv);
        F.rep0 = unii(rep0); F.rep1 = unii(rep1); F.rep2 = unii(rep2);
    } else if (p != be) {
        return ZC;
    }
    // last literals
    const int rem = rs - lp;
    if (rem > 0) {
        if (rem > fcs - op) return ZC;
        O.literals(lw, lsrc, lpos + lp, op, rem, lane);
        op += rem;
    }
    return op;
}

// one frame in rin[0, cs) -> out[0, cap): returns the decoded size or an error code
// lout: the output region for reading decoded literals back (whole dwords: its range ends at
// the dword holding the last byte, so no load that straddles the end reads back as zero)
__device__ __forceinline__ int decode_frame(const Bytes& rin, const Bytes& lout, int cs, ZSink& O, LDSA Lds& L, int cap,
                            int lane, unsigned long long* stats) {
    ZWin fw;
    fw.bind(rin, nullptr);
    fw.load(0, lane);
    if (cs < 9) return ZC;
    const uint32_t magic = fword(fw, 0, lane);
    if (magic != 0xFD2FB528u) return (magic & 0xFFFFFFF0u) == 0x184D2A50u ? kErrUnsupported : kErrCorrupt;
    const uint32_t fhd = fbyte(fw, 4, lane);
    const int fcsf = (int)(fhd >> 6), single = (int)((fhd >> 5) & 1u);
    if (fhd & 8u) return ZC;                  // reserved bit
    const int ccrc = (fhd & 4u) ? 4 : 0;      // content checksum: XXH64 low 32 bits after the last block
    int p = 5;
    if (!single) {
        const uint32_t wd = fbyte(fw, p++, lane);
        if ((wd >> 3) + 10 > 27) return kErrUnsupported;   // window beyond the reference's default limit
    }
    const int dsz = (int)(fhd & 3u) == 3 ? 4 : (int)(fhd & 3u);
    uint32_t dict = 0;
    for (int i = 0; i < dsz; i++) dict |= fbyte(fw, p + i, lane) << (8 * i);
    p += dsz;
    if (dict) return kErrUnsupported;
    const int fsz = fcsf == 0 ? (single ? 1 : 0) : (fcsf == 1 ? 2 : (fcsf == 2 ? 4 : 8));
    if (fsz == 0) return kErrUnsupported;              // content size absent
    uint64_t fcs = 0;
    for (int i = 0; i < fsz; i++) fcs |= (uint64_t)fbyte(fw, p + i, lane) << (8 * i);
    if (fsz == 2) fcs += 256;
    p += fsz;
    if (fcs > (uint64_t)cap) return ZC;
    const int n = (int)fcs;
    FrameState F{1, 4, 8, 0, 0, 0, false, false, false, false, false, 0, {0, 0, 0, 0, 0, 0, 0, 0}, 0};
    if (LZH_ZSTD_STATS) F.clk_last = __builtin_amdgcn_s_memtime();
    ZWin lw;
    lw.bind(rin, nullptr);
    lw.load(0, lane);
    int op = 0;
    for (int guard = 0; guard <= cs; guard++) {
        if (p + 3 > cs) return ZC;
        const uint32_t bh = fbyte(fw, p, lane) | (fbyte(fw, p + 1, lane) << 8) | (fbyte(fw, p + 2, lane) << 16);
        p += 3;
        const int last = (int)(bh & 1u), type = (int)((bh >> 1) & 3u), bsz = (int)(bh >> 3);
        if (bsz > kBlockMax) return ZC;
        if (type == 0) {
            if (p + bsz > cs || bsz > n - op) return ZC;
            O.literals(fw, rin, p, op, bsz, lane);
            op += bsz;
            p += bsz;
        } else if (type == 1) {
            if (p + 1 > cs || bsz > n - op) return ZC;
            const uint32_t v = fbyte(fw, p, lane);
            for (int base = 0; base < bsz; base += LZH_WAVE) {
                if (base + lane < bsz) O.put(op + base + lane, v);
                O.maybe_flush(op + min(base + LZH_WAVE, bsz), lane);
            }
            op += bsz;
            p += 1;
        } else if (type == 2) {
            if (p + bsz > cs) return ZC;
            const int r = decode_block(rin, lout, fw, lw, O, L, F, p, p + bsz, op, n, lane);
            if (r < 0) return r;
            op = r;
            p += bsz;
        } else {
            return ZC;
        }
        if (last) break;
    }
    ZCLK(F, 7);
    if (LZH_ZSTD_STATS && stats && lane == 0)
        for (int i = 0; i < kZClk; i++) atomicAdd(&stats[i], (unsigned long long)F.clk[i]);
    if (op != n || p + ccrc != cs) return ZC;
    if (ccrc) {   // ZSTD_decompressFrame's checksum check (zstd_decompress.c:1011-1020), once the output is out
        O.flush(op, lane);
        wait_vm();
        const uint32_t want = fword(fw, p, lane);
        if ((uint32_t)xxh64_wave(O.out, op, lane) != want) return kErrChecksum;
        O.flushed = op;
    }
    return op;
}

}  // namespace zstdd

// ---------------------------------------------------------------------------------------
// zstd decoding in three kernels.  The sequence section's decoding chain (bit reader, three FSE
// states, repcodes: ZSTD_decodeSequence, zstd_decompress_block.c:1169-1270) is serial within a
// block but independent between frames, so it runs one frame per LANE; what surrounds it is
// wave-parallel per frame:
//  1. lzh_zstd_hdr_kernel (one wave per frame): frame header, block walk, literal sections (the
//     Huffman streams decode into the frame's output tail), sequence-section headers; the FSE
//     tables it builds go to global memory per block.  Everything that does not need the output
//     position is checked here, in decode_frame's order.
//  2. lzh_zstd_seq_kernel (kFPW frames per wave, one per lane, tables in LDS): the sequences, with
//     every check of ZSTD_execSequence that depends on the output position; writes (ll, ml, offset)
//     per sequence.
//  3. lzh_zstd_exec_kernel (one wave per frame): executes them 64 at a time (groups::emit_group),
//     raw / RLE blocks and the content checksum.
// A frame that does not fit the layout (more blocks than bmax, more sequences than smax, a length
// of 2^17 or more) is decoded by lzh_zstd_decompress_kernel (the one-wave-per-frame decoder above)
// after the three.  Verdicts equal decode_frame's: every check is made, on the same quantities;
// only the order between checks differs, and every one of them reports kErrCorrupt.
//
// Literals of every block whose literal section is not raw live at the frame's output tail,
// block after block: [n - L, n) for L literals in all, so that the output of an accepted frame
// never overtakes a literal not yet copied (it holds every literal, and matches only add bytes).
namespace zsplit {
using namespace zstdd;

constexpr int kFPW = 8;              // frames per sequence-decoding wave (lanes 0 .. kFPW-1)
// the dummy stores' area after the frames' temp (512 bytes a sequence wave: a wave's lanes without a record
// store into their own wave's slice -- one shared slice for every wave was an L2 hot spot)
inline __host__ __device__ uint64_t zdummy_bytes(uint64_t nchunks) {   // (two launches' worth: see the launcher)
    const uint64_t w = (nchunks + kFPW - 1) / kFPW;
    return 2 * 512 * (w ? w : 1);
}
// A block's sequence tables in global memory (kSlot bytes): LL u32[512] | ML u32[512] | OF u16[256].
// LL / ML cell: next-state base (9) | nbBits << 9 (4) | extra bits << 13 (5) | pow << 18 | lo << 19
// (7): the baseline is lo, or 2^extra + lo for the codes whose baseline is >= 128 (LL 2^n, ML
// 2^n + 3): no baseline table on the chain.  OF cell (16 bits): e | code << 9 with e = 2 * base +
// 2^nbBits (a next-state base is a multiple of 2^nbBits: nbBits = ctz(e)).
constexpr int kSlot = 4608;
constexpr int kGo = 0, kLegacy = 1, kDone = 2;
constexpr int kLenBits = 17;         // (ll, ml, offset) packed as 17 + 17 + 30 bits

struct ZBlk {                        // a block of the frame (header kernel)
    uint32_t type;                   // 0 raw, 1 RLE, 2 compressed
    uint32_t ltype;                  // literals section type (compressed blocks)
    uint32_t pos;                    // raw: data position in the frame; RLE: the byte; else sequence stream start
    uint32_t size;                   // raw / RLE: block size; else sequence stream bytes
    uint32_t rs;                     // literals
    uint32_t lit;                    // literals' position: ltype 0 in the frame, else in the output
    uint32_t nseq;
    uint32_t logs;                   // accuracy logs LL | OF << 8 | ML << 16
    uint32_t tll, tof, tml;          // the blocks (of this frame) whose table slots hold LL / OF / ML
    uint32_t pad;
};
// blocks, content size, checksum position (-1: none); sv: the sequence kernel's verdict (kGo, kLegacy or
// an error), applied by the execution kernel -- the sequence kernel runs beside the literal kernels, which
// write zst / status themselves, and their verdict comes first
struct ZFrame { int32_t nblk, n, ccrc, sv, nsq, pad0, pad1, pad2; };   // (nsq: the frame's sequences)
struct ZExe { uint32_t op0, seq0; };             // a block's output position and first sequence
// a Huffman-coded literal section (header kernel -> literal kernel): its frame, the block whose
// table slot holds its table, the table log, whether the reference would decode it with the
// double-symbol decoder, streams, output position, symbols per stream (the 4th: last), streams
constexpr int kHufSlot = 4096;                   // a table of up to 2^11 16-bit cells (symbol | nbBits << 8)
struct ZHuf {
    uint32_t frame, tblk, tl, x2, ns, dst, seg, last;
    uint32_t s0[4], sz[4];
};

struct ZLayout {
    uint64_t bmax, smax, stride;
    __host__ __device__ uint64_t exe() const { return bmax * sizeof(ZBlk); }
    __host__ __device__ uint64_t cells() const { return exe() + bmax * sizeof(ZExe); }
    __host__ __device__ uint64_t hufs() const { return cells() + bmax * kSlot; }
    __host__ __device__ uint64_t seqs() const { return hufs() + bmax * kHufSlot; }
};
__host__ __device__ inline ZLayout zlayout(uint64_t chunk) {
    ZLayout L;
    L.bmax = (chunk + kBlockMax - 1) / kBlockMax + 1;   // the compressor writes ceil(chunk / 128 KiB) blocks
    L.smax = chunk / 4 + 64;                            // (its matches are >= 4 bytes)
    L.stride = (L.seqs() + L.smax * 8 + 255) & ~255ull;
    return L;
}

// one compressed block's literal section and sequence-section header (decode_block up to the
// sequences); lacc = the next literal position at the output tail
__device__ __forceinline__ int hdr_block(const Bytes& rin, const Bytes& rout, ZWin& fw, LDSA Lds& L, FrameState& F,
                                         int bs, int be, int& lacc, ZBlk& B, uint8_t* cells, int b, int& tll, int& tof,
                                         int& tml, int& thuf, uint8_t* hufs, ZHuf* jobs, uint32_t* njobs, uint32_t frame,
                                         int lane) {
    const uint32_t b0 = fbyte(fw, bs, lane);
    const int ltype = (int)(b0 & 3u), sf = (int)((b0 >> 2) & 3u);
    int rs, seqpos;
    if (ltype <= 1) {
        int hsz;
        if ((sf & 1) == 0) { hsz = 1; rs = (int)(b0 >> 3); }
        else if (sf == 1) { hsz = 2; rs = (int)((b0 >> 4) + (fbyte(fw, bs + 1, lane) << 4)); }
        else { hsz = 3; rs = (int)((b0 >> 4) + (fbyte(fw, bs + 1, lane) << 4) + (fbyte(fw, bs + 2, lane) << 12)); }
        if (rs > kBlockMax) return ZC;
        if (ltype == 0) {
            if (bs + hsz + rs > be) return ZC;
            B.lit = (uint32_t)(bs + hsz);
            seqpos = bs + hsz + rs;
        } else {
            if (bs + hsz + 1 > be) return ZC;   // (rs > fcs - op: the sequence kernel)
            const uint32_t v = fbyte(fw, bs + hsz, lane);
            for (int i = lane; i < rs; i += LZH_WAVE) rout.st8(lacc + i, v);
            B.lit = (uint32_t)lacc;
            lacc += rs;
            seqpos = bs + hsz + 1;
        }
    } else {
        const int hsz = sf <= 1 ? 3 : (sf == 2 ? 4 : 5);
        const int bits = sf <= 1 ? 10 : (sf == 2 ? 14 : 18);
        if (bs + hsz > be) return ZC;
        uint64_t h = 0;
        for (int i = 0; i < hsz; i++) h |= (uint64_t)fbyte(fw, bs + i, lane) << (8 * i);
        rs = (int)((h >> 4) & ((1u << bits) - 1));
        const int cs = (int)((h >> (4 + bits)) & ((1u << bits) - 1));
        if (rs > kBlockMax || bs + hsz + cs > be) return ZC;
        int p = bs + hsz;
        if (ltype == 2) {
            int tl = 0;
            ZCLK(F, 0);
            const int u = read_huf(fw, rin, p, bs + hsz + cs, L, tl, lane);
            ZCLK(F, 1);
            if (u < 0) return u;
            F.hufV = true;
            F.hufTl = tl;
            F.hufX2 = sf != 0 && huf_select_x2(rs, cs);
            p += u;
        } else if (!F.hufV) {
            return ZC;
        }
        if (rs == 0 && sf != 0 && ltype == 2) return ZC;
        if (F.hufTl > 11) return kLegacy;            // (the literal kernel's table slots hold 2^11 cells)
        if (ltype == 2) {                            // the table to the block's slot
            uint32_t* dst = (uint32_t*)(hufs + (size_t)b * kHufSlot);
            const LDSA uint32_t* src = (const LDSA uint32_t*)L.huf;
            for (int c = lane; c < (1 << F.hufTl) / 2; c += LZH_WAVE) dst[c] = src[c];
            thuf = b;
        }
        // the streams' geometry and end marks, as huf_streams checks them; the literal kernel decodes
        const int csize = bs + hsz + cs - p, ns = sf == 0 ? 1 : 4;
        ZHuf J{};
        J.frame = frame;
        J.tblk = (uint32_t)thuf;
        J.tl = (uint32_t)F.hufTl;
        J.x2 = F.hufX2 ? 1u : 0u;
        J.ns = (uint32_t)ns;
        J.dst = (uint32_t)lacc;
        if (ns == 4) {
            if (csize < 10) return ZC;
            const int z1 = (int)(fword(fw, p, lane) & 0xffffu), z2 = (int)(fword(fw, p + 2, lane) & 0xffffu),
                      z3 = (int)(fword(fw, p + 4, lane) & 0xffffu);
            const int z4 = csize - 6 - z1 - z2 - z3;
            if (z4 < 1) return ZC;
            const int seg = (rs + 3) / 4, last = rs - 3 * seg;
            if (last < 0) return ZC;
            if (z1 <= 0 || z2 <= 0 || z3 <= 0) return ZC;
            J.seg = (uint32_t)seg;
            J.last = (uint32_t)last;
            const int p1 = p + 6;
            J.s0[0] = (uint32_t)p1; J.s0[1] = (uint32_t)(p1 + z1); J.s0[2] = (uint32_t)(p1 + z1 + z2);
            J.s0[3] = (uint32_t)(p1 + z1 + z2 + z3);
            J.sz[0] = (uint32_t)z1; J.sz[1] = (uint32_t)z2; J.sz[2] = (uint32_t)z3; J.sz[3] = (uint32_t)z4;
        } else {
            if (csize <= 0) return ZC;
            J.seg = J.last = (uint32_t)rs;
            J.s0[0] = (uint32_t)p;
            J.sz[0] = (uint32_t)csize;
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (k < ns && fbyte(fw, (int)(J.s0[k] + J.sz[k]) - 1, lane) == 0) return ZC;   // (BIT_initDStream: no end mark)
        if (lane == 0) jobs[atomicAdd(njobs, 1u)] = J;
        B.lit = (uint32_t)lacc;
        lacc += rs;
        seqpos = bs + hsz + cs;
    }
    B.ltype = (uint32_t)ltype;
    B.rs = (uint32_t)rs;
    // sequences section header (ZSTD_decodeSeqHeaders)
    if (seqpos >= be) return ZC;
    int p = seqpos;
    int nseq = (int)fbyte(fw, p++, lane);
    if (nseq >= 128) {
        if (nseq == 255) {
            if (p + 2 > be) return ZC;
            nseq = (int)(fbyte(fw, p, lane) + (fbyte(fw, p + 1, lane) << 8)) + 0x7F00;
            p += 2;
        } else {
            if (p + 1 > be) return ZC;
            nseq = ((nseq - 128) << 8) + (int)fbyte(fw, p++, lane);
        }
    }
    B.nseq = (uint32_t)nseq;
    if (nseq > 0) {
        if (p >= be) return ZC;
        const uint32_t modes = fbyte(fw, p++, lane);
        if (modes & 3u) return ZC;
        // a table built in this block goes to the block's slot; "repeat" keeps the previous slot
        auto table = [&](int mode, int which, LDSA Cell* T, int& al, bool& valid, int& slot) -> bool {
            const int u = seq_table(fw, p, be, mode, which, T, al, valid, L, lane);
            if (u < 0) return false;
            p += u;
            if (mode != 3) {   // the cells in the sequence kernel's formats (kSlot)
                uint8_t* dst = cells + (size_t)b * kSlot;
                for (int c = lane; c < (1 << al); c += LZH_WAVE) {
                    const Cell e = T[c];
                    const uint32_t nx = c_next(e), nb = (uint32_t)c_nb(e), add = (uint32_t)c_add(e), sym = c_sym(e);
                    if (which == 1) {
                        ((uint16_t*)(dst + 4096))[c] = (uint16_t)((2u * nx + (1u << nb)) | (sym << 9));
                    } else {
                        const uint32_t base = which == 0 ? kLLBase[sym] : kMLBase[sym];
                        const uint32_t pw = base >= 128u;
                        const uint32_t lo = pw ? base - (1u << add) : base;
                        ((uint32_t*)(dst + (which == 0 ? 0 : 2048)))[c] = nx | (nb << 9) | (add << 13) | (pw << 18) | (lo << 19);
                    }
                }
                slot = b;
            }
            return true;
        };
        ZCLK(F, 0);
        if (!table((int)(modes >> 6), 0, L.ll, F.llA, F.llV, tll)) return ZC;
        if (!table((int)((modes >> 4) & 3u), 1, L.of, F.ofA, F.ofV, tof)) return ZC;
        if (!table((int)((modes >> 2) & 3u), 2, L.ml, F.mlA, F.mlV, tml)) return ZC;
        ZCLK(F, 3);
        B.logs = (uint32_t)F.llA | ((uint32_t)F.ofA << 8) | ((uint32_t)F.mlA << 16);
        B.tll = (uint32_t)tll; B.tof = (uint32_t)tof; B.tml = (uint32_t)tml;
        B.pos = (uint32_t)p;
        B.size = (uint32_t)(be - p);
    } else if (p != be) {
        return ZC;
    }
    return 0;
}

// the frame's header and blocks (decode_frame without the sequences); returns kGo / kLegacy or an error
__device__ __forceinline__ int hdr_frame_body(const Bytes& rin, const Bytes& rout, int cs, LDSA Lds& L, int cap,
                                              uint8_t* zb, const ZLayout& Z, ZFrame& fr, int lane, FrameState& F,
                                              ZHuf* jobs, uint32_t* njobs, uint32_t frame) {
    ZWin fw;
    fw.bind(rin, nullptr);
    fw.load(0, lane);
    if (cs < 9) return ZC;
    const uint32_t magic = fword(fw, 0, lane);
    if (magic != 0xFD2FB528u) return (magic & 0xFFFFFFF0u) == 0x184D2A50u ? kErrUnsupported : kErrCorrupt;
    const uint32_t fhd = fbyte(fw, 4, lane);
    const int fcsf = (int)(fhd >> 6), single = (int)((fhd >> 5) & 1u);
    if (fhd & 8u) return ZC;
    const int ccrc = (fhd & 4u) ? 4 : 0;
    int p = 5;
    if (!single) {
        const uint32_t wd = fbyte(fw, p++, lane);
        if ((wd >> 3) + 10 > 27) return kErrUnsupported;
    }
    const int dsz = (int)(fhd & 3u) == 3 ? 4 : (int)(fhd & 3u);
    uint32_t dict = 0;
    for (int i = 0; i < dsz; i++) dict |= fbyte(fw, p + i, lane) << (8 * i);
    p += dsz;
    if (dict) return kErrUnsupported;
    const int fsz = fcsf == 0 ? (single ? 1 : 0) : (fcsf == 1 ? 2 : (fcsf == 2 ? 4 : 8));
    if (fsz == 0) return kErrUnsupported;
    uint64_t fcs = 0;
    for (int i = 0; i < fsz; i++) fcs |= (uint64_t)fbyte(fw, p + i, lane) << (8 * i);
    if (fsz == 2) fcs += 256;
    p += fsz;
    if (fcs > (uint64_t)cap) return ZC;
    const int n = (int)fcs;
    // walk the block headers and literal-section sizes first: the tail layout needs the total
    int nb = 0, ltot = 0;
    {
        int q = p;
        for (int guard = 0; guard <= cs; guard++) {
            if (q + 3 > cs) return ZC;
            const uint32_t bh = fbyte(fw, q, lane) | (fbyte(fw, q + 1, lane) << 8) | (fbyte(fw, q + 2, lane) << 16);
            q += 3;
            const int last = (int)(bh & 1u), type = (int)((bh >> 1) & 3u), bsz = (int)(bh >> 3);
            if (bsz > kBlockMax) return ZC;
            if (++nb > (int)Z.bmax) return kLegacy;
            if (type == 0) {
                if (q + bsz > cs) return ZC;
                q += bsz;
            } else if (type == 1) {
                if (q + 1 > cs) return ZC;
                q += 1;
            } else if (type == 2) {
                if (q + bsz > cs || bsz < 1) return ZC;
                const uint32_t b0 = fbyte(fw, q, lane);
                const int ltype = (int)(b0 & 3u), sf = (int)((b0 >> 2) & 3u);
                int rs;
                if (ltype <= 1) {
                    const int hsz = (sf & 1) == 0 ? 1 : (sf == 1 ? 2 : 3);
                    if (q + hsz > cs) return ZC;
                    rs = (sf & 1) == 0 ? (int)(b0 >> 3)
                                       : (sf == 1 ? (int)((b0 >> 4) + (fbyte(fw, q + 1, lane) << 4))
                                                  : (int)((b0 >> 4) + (fbyte(fw, q + 1, lane) << 4) +
                                                          (fbyte(fw, q + 2, lane) << 12)));
                } else {
                    const int hsz = sf <= 1 ? 3 : (sf == 2 ? 4 : 5);
                    const int bits = sf <= 1 ? 10 : (sf == 2 ? 14 : 18);
                    if (hsz > bsz) return ZC;
                    uint64_t h = 0;
                    for (int i = 0; i < hsz; i++) h |= (uint64_t)fbyte(fw, q + i, lane) << (8 * i);
                    rs = (int)((h >> 4) & ((1u << bits) - 1));
                }
                if (rs > kBlockMax) return ZC;
                if (ltype != 0) ltot += rs;
                q += bsz;
            } else {
                return ZC;
            }
            if (last) break;
        }
    }
    if (ltot > n) return ZC;   // an accepted frame's output holds every literal
    ZBlk* blk = (ZBlk*)zb;
    uint8_t* cells = zb + Z.cells();
    int lacc = n - ltot, tll = 0, tof = 0, tml = 0, thuf = 0, nsq = 0;
    for (int b = 0; b < nb; b++) {
        const uint32_t bh = fbyte(fw, p, lane) | (fbyte(fw, p + 1, lane) << 8) | (fbyte(fw, p + 2, lane) << 16);
        p += 3;
        const int type = (int)((bh >> 1) & 3u), bsz = (int)(bh >> 3);
        ZBlk B{};
        B.type = (uint32_t)type;
        if (type == 0) {
            B.pos = (uint32_t)p;
            B.size = (uint32_t)bsz;
            p += bsz;
        } else if (type == 1) {
            B.pos = fbyte(fw, p, lane);
            B.size = (uint32_t)bsz;
            p += 1;
        } else {
            const int r = hdr_block(rin, rout, fw, L, F, p, p + bsz, lacc, B, cells, b, tll, tof, tml, thuf, zb + Z.hufs(),
                                    jobs, njobs, frame, lane);
            if (r != 0) return r;   // (an error, or kLegacy)
            p += bsz;
            nsq += (int)B.nseq;
        }
        if (lane == 0) blk[b] = B;
    }
    if (p + ccrc != cs) return ZC;
    fr.nsq = nsq;
    fr.nblk = nb;
    fr.n = n;
    fr.ccrc = ccrc ? p : -1;
    return kGo;
}

__device__ __forceinline__ int hdr_frame(const Bytes& rin, const Bytes& rout, int cs, LDSA Lds& L, int cap, uint8_t* zb,
                                         const ZLayout& Z, ZFrame& fr, int lane, unsigned long long* stats, ZHuf* jobs,
                                         uint32_t* njobs, uint32_t frame) {
    FrameState F{1, 4, 8, 0, 0, 0, false, false, false, false, false, 0, {0, 0, 0, 0, 0, 0, 0, 0}, 0};
    if (LZH_ZSTD_STATS) F.clk_last = __builtin_amdgcn_s_memtime();
    const int r = hdr_frame_body(rin, rout, cs, L, cap, zb, Z, fr, lane, F, jobs, njobs, frame);
    ZCLK(F, 7);
    if (LZH_ZSTD_STATS && stats && lane == 0)
        for (int i = 0; i < kZClk; i++) atomicAdd(&stats[i], (unsigned long long)F.clk[i]);
    return r;
}

// The sequence kernel's LDS (kFPW lanes; a "row" holds one dword per lane, as an LDS-DMA
// (global_load_lds_dword) writes it: lane i at row + 4 i): LL cells 512 rows, ML 512, OF 128 (two
// 16-bit cells a dword), the bit-stream ring (64 rows: stream dword d at row d mod 64, two halves of
// 32-dword blocks, + a mirror of row 0), the sequences buffered between flush points (kSB per lane,
// 8 bytes).  39 456 bytes: 4 waves per CU.
constexpr int kRow = 4 * kFPW;
constexpr int kSB = 16;                         // steps between flush / fill points
constexpr int kLdsML = 512 * kRow, kLdsOF = 1024 * kRow, kLdsRing = 1152 * kRow, kLdsSB = 1217 * kRow;
constexpr int kLdsSeq = kLdsSB;

__device__ __forceinline__ void dma_row(const uint8_t* src, LDSA uint8_t* row) {
    __builtin_amdgcn_global_load_lds((const void*)src, (LDSA void*)row, 4, 0, 0);
}
// s_waitcnt immediate for vmcnt(n) alone (gfx9: vmcnt bits [3:0] and [15:14], expcnt / lgkmcnt at max)
constexpr int vmcnt_imm(int n) { return 0x0F70 | (n & 15) | ((n >> 4) << 14); }
// one dword per lane from a buffer resource into an LDS row (out-of-range offsets read 0, so a
// negative or oversized per-lane offset needs no clamp).  (No instruction offset: an LDS-DMA adds it
// to the LDS address as well.)
__device__ __forceinline__ void dma_rs(rsrc_t r, LDSA uint8_t* row, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (LDSA void*)row, 4, voff, 0, 0, 0);
}
// a buffer resource over [base, base + bytes), bytes clamped to the 32-bit record count
__device__ __forceinline__ rsrc_t rsrc_over(const void* base, uint64_t bytes) {
    return make_rsrc(base, (uint32_t)min<uint64_t>(bytes, 0xffffffffull));
}

// c ? a : b as one v_cndmask on the condition's lane mask (no branch)
__device__ __forceinline__ int vsel(bool c, int a, int b) {
    int r;
    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(r) : "v"(b), "v"(a), "s"(__builtin_amdgcn_ballot_w64(c)));
    return r;
}

}  // namespace zsplit

// Sequences, one frame per lane (lanes 0 .. kFPW-1), in lock-step steps of one sequence per lane:
// ZSTD_decodeSequence (zstd_decompress_block.c:1169-1270) with the FSE tables and the bit stream in
// LDS, and every check of ZSTD_execSequence that depends on the output position (decode_block's).
// A step reads the three cells, then the sequence's four bit fields at once (offset extra bits, match
// and literal length extra bits, the three state updates: their widths are known from the cells, so
// are the positions) -- two LDS round trips per sequence, no bit container.  The steps run in
// intervals of kSB; between intervals (a uniform point, all lanes): wait for the memory operations
// issued before, flush the buffered sequences, mark the fills issued at the previous point ready,
// start blocks (raw / RLE / empty ones pass through), give the upper ring block back once the reader
// is below it, issue the fills lanes asked for -- a block's tables and 32-dword stream blocks -- as
// LDS-DMA rows masked to those lanes (no load result passes through registers: a per-lane register
// prefetch would be waited for at once, the wave's memory counter does not tell lanes apart), and
// set each lane's lowest safe position (the ready data must cover the <= 90 bits a sequence reads).
// A wave issues one instruction per 4 cycles whatever its lanes do, so the step is kept lean: no
// branches but the skip and the block's end.
extern "C" __global__ void __launch_bounds__(64)
lzh_zstd_seq_kernel(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets, uint64_t chunk_size,
                    uint32_t nchunks, int32_t* status, uint8_t* zt, const int32_t* zst, zsplit::ZFrame* zfr,
                    unsigned long long* stats, const uint32_t* flist, const uint32_t* fcnt, int which) {
    using namespace zsplit;
    using namespace zstdd;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsSeq];
    LDSA uint8_t* const S = (LDSA uint8_t*)lds;
    const int lane = threadIdx.x;
    // (the chain of one wave per SIMD is the kernel's time: its instructions go first when other kernels' waves
    // -- the literal and execution kernels beside it -- share its SIMD)
    __builtin_amdgcn_s_setprio(3);
    // frames: lane of wave blockIdx.x, or (which 0 / 1) entry of the planned short list (from the front) /
    // long list (from the back) -- lzh_zstd_plan_kernel
    const uint32_t x = blockIdx.x * kFPW + (uint32_t)lane;
    const bool inl = lane < kFPW && (which < 0 ? x < nchunks : x < fcnt[which]);
    const uint32_t f = !inl ? 0u : which < 0 ? x : (which == 0 ? flist[x] : flist[nchunks - 1 - x]);
    const bool live = inl && zst[f] == kGo;
    const ZLayout Z = zlayout(chunk_size);
    uint8_t* const zb = zt + (uint64_t)(live ? f : 0) * Z.stride;
    const ZBlk* blk = (const ZBlk*)zb;
    ZExe* ex = (ZExe*)(zb + Z.exe());
    uint64_t* seqs = (uint64_t*)(zb + Z.seqs());
    int nblk = 0, n = 0;
    int64_t ioff = 0;
    if (live) {
        const ZFrame fr = zfr[f];
        nblk = fr.nblk;
        n = fr.n;
        ioff = (int64_t)offsets[f];
    }
    // (fills are global_load_lds rows from per-lane addresses: with a buffer resource the kernel's
    // scalar-register pressure moved it to vector registers and every fill became a waterfall loop)
    const int64_t readable = (int64_t)packed_readable;
    uint64_t* const dummy = (uint64_t*)(zt + (uint64_t)nchunks * Z.stride) +
                            64ull * (blockIdx.x + (which == 1 ? gridDim.x : 0u));   // (the wave's slice)
    const int lo4 = lane * 4;
    int phase = live ? 0 : 3, res = kGo;   // 0 block start, 1 waiting for fills, 2 sequences, 3 finished
    int b = 0, op = 0, rep0 = 1, rep1 = 4, rep2 = 8;
    uint32_t sfl = 0;                                           // sequences stored
    int rs = 0, lp = 0, nseq = 0, i = 0, lA = 0, oA = 0, mA = 0;
    uint32_t sLL = 0, sOF = 0, sML = 0;
    const uint8_t *tLL = zb, *tOF = zb, *tML = zb;   // the block's table slots
    int64_t A = 0;                       // the stream's first byte rounded down to a dword (absolute)
    int P = 0, lo = 0;                   // bits [lo, P) of the stream are unread (positions from A)
    int hb0 = 0, hb1 = 0;                // the 32-dword stream blocks in ring halves 0 / 1
    int rdy = 0, req = 0, iss = 0;       // halves ready / requested / in flight (bits 0, 1)
    int lowok = 1 << 30;                 // a step runs while P >= lowok
    bool treq = false, tiss = false, trdy = false;
    const int smax = (int)Z.smax;

    // bits [q, q + w) of the stream (w <= 31): rows of dwords q / 32 and the one above, a funnel
    // shift and a bit-field extract
    auto fld = [&](int q, int w) -> uint32_t {
        const LDSA uint8_t* a = S + kLdsRing + ((q >> 5) & 63) * kRow + lo4;
        const uint32_t v = __builtin_amdgcn_alignbit(*(const LDSA uint32_t*)(a + kRow), *(const LDSA uint32_t*)a,
                                                     (uint32_t)q & 31u);
        return __builtin_amdgcn_ubfe(v, 0u, (uint32_t)w);
    };

    // every step stores one record per lane at seqp[sfl] and advances sfl when the record is kept: a lane
    // without one writes the slot its next record overwrites (or the spare slot past its last), a lane
    // without a frame its own word of the wave's dummy slice (its sfl stays 0)
    uint64_t* const seqp = live ? seqs : dummy + lane;
    // (the lane's column of the bit ring, opaque to the compiler: it would split the ring's offset back out
    // and add it per address, the ds_read2 offset field being too small for it)
    const LDSA uint8_t* rb = S + kLdsRing + lo4;
    asm volatile("" : "+v"(rb));
    uint64_t sst[6] = {0, 0, 0, 0, 0, 0}, tmark = 0;   // (LZH_ZSTD_STATS: uniform points, steps, ...)
    const uint64_t tm0 = LZH_ZSTD_STATS ? __builtin_amdgcn_s_memtime() : 0, tr0 = LZH_ZSTD_STATS ? __builtin_amdgcn_s_memrealtime() : 0;
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): the compiler's own wait tracking sees it
    for (int ival = 0;; ival++) {
        if (LZH_ZSTD_STATS) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            if (ival) sst[1] += t - tmark;
            tmark = t;
            sst[2]++;
        }
        // ---- uniform point
        // every memory operation but the previous point's kSB flush stores (issued after its fills) is done
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(kSB));
        if (LZH_ZSTD_STATS) sst[5] += __builtin_amdgcn_s_memtime() - tmark;
        rdy |= iss;
        iss = 0;
        if (tiss) { tiss = false; trdy = true; }
        if (phase == 1 && trdy && rdy == 3) {   // the block's first states (LL, OF, ML)
            sLL = fld(P - lA, lA);
            sOF = fld(P - lA - oA, oA);
            sML = fld(P - lA - oA - mA, mA);
            P -= lA + oA + mA;
            phase = 2;
        }
        if (LZH_ZSTD_STATS) sst[3] += ballot(phase == 0) != 0;
        while (phase == 0) {   // the next blocks, up to one with sequences (or the end of the frame)
            if (b == nblk) {
                if (op != n) res = ZC;
                phase = 3;
                break;
            }
            const ZBlk B = blk[b];
            const int si = sfl;
            if (B.type != 2) {
                if ((int)B.size > n - op) { res = ZC; phase = 3; break; }
                ex[b] = ZExe{(uint32_t)op, (uint32_t)si};
                op += (int)B.size;
                b++;
                continue;
            }
            rs = (int)B.rs;
            if (B.ltype != 0 && rs > n - op) { res = ZC; phase = 3; break; }
            ex[b] = ZExe{(uint32_t)op, (uint32_t)si};
            lp = 0;
            i = 0;
            nseq = (int)B.nseq;
            b++;
            if (nseq == 0) {
                if (rs > n - op) { res = ZC; phase = 3; break; }
                op += rs;
                continue;
            }
            if ((int)sfl + nseq > smax - 1) { res = kLegacy; phase = 3; break; }   // (the layout's record slots, one spare)
            lA = (int)(B.logs & 255u);
            oA = (int)((B.logs >> 8) & 255u);
            mA = (int)(B.logs >> 16);
            const uint8_t* cz = zb + Z.cells();
            tLL = cz + (size_t)B.tll * kSlot;
            tML = cz + (size_t)B.tml * kSlot + 2048;
            tOF = cz + (size_t)B.tof * kSlot + 4096;
            treq = true;
            trdy = false;
            // the stream's end mark (BIT_initDStream) and the two blocks below it
            const int64_t s0 = ioff + (int64_t)B.pos;
            const int size = (int)B.size;
            if (size <= 0) { res = ZC; phase = 3; break; }
            A = s0 & ~3ll;
            const int x0 = (int)(s0 & 3), X = x0 + size - 1;
            const uint32_t last = packed[A + X];
            if (last == 0) { res = ZC; phase = 3; break; }
            lo = 8 * x0;
            P = 8 * X + hb32(last);
            const int bt = (P - 1) >> 10;
            hb0 = (bt & 1) ? bt - 1 : bt;
            hb1 = (bt & 1) ? bt : bt - 1;
            rdy = 0;
            iss = 0;
            req = 3;
            phase = 1;
        }
        if (phase == 2) {   // the upper block, once the reader is below it, takes the block under the lower one
            const int top = (P - 1) >> 10;
            const bool r0 = (rdy & 1) != 0 && hb0 > top && hb0 > hb1, r1 = (rdy & 2) != 0 && hb1 > top && hb1 > hb0;
            if (r0) { hb0 = hb1 - 1; rdy &= ~1; req |= 1; }
            if (r1) { hb1 = hb0 - 1; rdy &= ~2; req |= 2; }
        }
        if (ballot(treq)) {
            if (treq) {
#pragma unroll 8
                for (int r = 0; r < 512; r++) dma_row(tLL + 4 * r, S + r * kRow);
#pragma unroll 8
                for (int r = 0; r < 512; r++) dma_row(tML + 4 * r, S + kLdsML + r * kRow);
#pragma unroll 8
                for (int r = 0; r < 128; r++) dma_row(tOF + 4 * r, S + kLdsOF + r * kRow);
                treq = false;
                tiss = true;
            }
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if (ballot(req & (1 << h))) {
                const int64_t x0 = A + 128ll * (h ? hb1 : hb0);
                // a block wholly outside the packed bytes holds no stream data: any readable bytes will do
                const bool part = x0 >= 0 && x0 < readable && x0 + 128 > readable;
                const uint8_t* g = packed + (x0 < 0 || x0 >= readable ? 0 : x0);
                if ((req & (1 << h)) && !part) {
#pragma unroll
                    for (int k = 0; k < 32; k++) dma_row(g + 4 * k, S + kLdsRing + (h * 32 + k) * kRow);
                    if (h == 0) dma_row(g, S + kLdsRing + 64 * kRow);   // (the mirror of row 0)
                }
                if (ballot((req & (1 << h)) && part)) {   // (the packed bytes end inside the block)
                    if ((req & (1 << h)) && part) {
                        for (int k = 0; k < 32; k++)
                            dma_row(packed + (x0 + 4 * k < readable - 4 ? x0 + 4 * k : ((readable - 4) & ~3ll)), S + kLdsRing + (h * 32 + k) * kRow);
                        if (h == 0) dma_row(packed + x0, S + kLdsRing + 64 * kRow);
                    }
                }
                if (req & (1 << h)) {
                    req &= ~(1 << h);
                    iss |= 1 << h;
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
        // the lowest position a step may start from: the ready blocks below the reader + 90 bits
        lowok = (rdy == 3 ? 1024 * min(hb0, hb1) : (rdy == 1 ? 1024 * hb0 : (rdy == 2 ? 1024 * hb1 : (1 << 30)))) + 90;
        if (phase != 2) lowok = 1 << 30;
        if (LZH_ZSTD_STATS) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            sst[0] += t - tmark;
            tmark = t;
        }
        if (!ballot(phase != 3)) break;
        if (ival > (smax + 64 * (int)Z.bmax) / 2) {   // (a bound every lane meets: a stuck lane's frame goes to
            if (phase != 3) { res = kLegacy; phase = 3; }   // the one-wave decoder)
            lowok = 1 << 30;
        }
        // the cells of the states (read one step ahead from here on: a step reads the next step's cells
        // as soon as its states are known, under its checks and record)
        uint32_t cL = 0, cM = 0, cO = 0;
        if (phase == 2) {
            cL = *(const LDSA uint32_t*)(S + sLL * kRow + lo4);
            cM = *(const LDSA uint32_t*)(S + kLdsML + sML * kRow + lo4);
            cO = *(const LDSA uint16_t*)(S + kLdsOF + (sOF >> 1) * kRow + lo4 + (sOF & 1) * 2);
        }
        // ---- kSB steps: each stores exactly one record per lane (a dummy word for a lane without one),
        // so that the next point's vmcnt(kSB) waits for this point's fills and not for these stores
        for (int k = 0; k < kSB; k++) {
            const bool act = P >= lowok;
            uint32_t r0 = 0, r1 = 0;
            bool keep = false;
            if (act) {
                const uint32_t eL = cL, eM = cM, eO = cO;
                const int ofc = (int)(eO >> 9);
                const uint32_t eOx = eO & 511u;
                const int no = (int)__builtin_ctz(eOx);
                const int am = (int)__builtin_amdgcn_ubfe(eM, 13u, 5u), al = (int)__builtin_amdgcn_ubfe(eL, 13u, 5u);
                const int nl = (int)__builtin_amdgcn_ubfe(eL, 9u, 4u), nm = (int)__builtin_amdgcn_ubfe(eM, 9u, 4u);
                const int ns = nl + nm + no;
                const bool lastq = i + 1 == nseq;
                // the fields: offset extra bits, ML extra bits, LL extra bits, LL / ML / OF state bits
                const int P1 = P - ofc, P2 = P1 - am, P3 = P2 - al, P4 = P3 - (lastq ? 0 : ns);
                // (the eight ring loads issued together, then used: the scheduler would wait after each pair)
                const LDSA uint8_t* a1 = rb + ((P1 >> 5) & 63) * kRow;
                const LDSA uint8_t* a2 = rb + ((P2 >> 5) & 63) * kRow;
                const LDSA uint8_t* a3 = rb + ((P3 >> 5) & 63) * kRow;
                const LDSA uint8_t* a4 = rb + ((P4 >> 5) & 63) * kRow;
                const uint32_t w1l = *(const LDSA uint32_t*)a1, w1h = *(const LDSA uint32_t*)(a1 + kRow);
                const uint32_t w2l = *(const LDSA uint32_t*)a2, w2h = *(const LDSA uint32_t*)(a2 + kRow);
                const uint32_t w3l = *(const LDSA uint32_t*)a3, w3h = *(const LDSA uint32_t*)(a3 + kRow);
                const uint32_t w4l = *(const LDSA uint32_t*)a4, w4h = *(const LDSA uint32_t*)(a4 + kRow);
                __builtin_amdgcn_sched_barrier(0);
                const uint32_t ob = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(w1h, w1l, (uint32_t)P1 & 31u), 0u, (uint32_t)ofc);
                const uint32_t mb = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(w2h, w2l, (uint32_t)P2 & 31u), 0u, (uint32_t)am);
                const uint32_t lb = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(w3h, w3l, (uint32_t)P3 & 31u), 0u, (uint32_t)al);
                const uint32_t sb = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(w4h, w4l, (uint32_t)P4 & 31u), 0u,
                                                          (uint32_t)(lastq ? 0 : ns));
                const int ml = (int)((__builtin_amdgcn_ubfe(eM, 18u, 1u) << am) + (eM >> 19) + mb);
                const int ll = (int)((__builtin_amdgcn_ubfe(eL, 18u, 1u) << al) + (eL >> 19) + lb);
                // repcodes (ZSTD_decodeSequence): ofc > 1 a new offset; else repcode j = ofc + ll0 + bit
                // (selects on lane masks: the compiler would branch on them)
                const bool big = ofc > 1;
                const int j = ofc + (int)((eL >> 18) == 0) + (int)ob;
                int t = vsel(j == 0, rep0, vsel(j == 1, rep1, vsel(j == 2, rep2, rep0 - 1)));
                t += t == 0;
                const int off = vsel(big, (int)((1u << ofc) - 3u + ob), t);
                const int nrep1 = vsel(big | (j >= 1), rep0, rep1);
                rep2 = vsel(big | (j >= 2), rep1, rep2);
                rep1 = nrep1;
                rep0 = off;
                sLL = (eL & 511u) + (sb >> (nm + no));
                sML = (eM & 511u) + __builtin_amdgcn_ubfe(sb, (uint32_t)no, (uint32_t)nm);
                sOF = ((eOx - (1u << no)) >> 1) + __builtin_amdgcn_ubfe(sb, 0u, (uint32_t)no);
                P = P4;
                cL = *(const LDSA uint32_t*)(S + sLL * kRow + lo4);
                cM = *(const LDSA uint32_t*)(S + kLdsML + sML * kRow + lo4);
                cO = *(const LDSA uint16_t*)(S + kLdsOF + (sOF >> 1) * kRow + lo4 + (sOF & 1) * 2);
                // the checks of ZSTD_execSequence and the layout's limit (else the one-wave decoder decodes).
                // Per step only the offset and the record width: the stream position only falls and the
                // literals used / the output plus the literals left only grow, so the checks on those hold
                // at every sequence of a block exactly when they hold at its last -- that is where they are
                // made (with the reference's end of stream: it updates the states after the last sequence too
                // and accepts an exhausted or overrun stream there, ZSTD_decompressSequences_body: reload >=
                // completed).  A frame that fails is not executed, so nothing reads the records before it.
                const bool bad = (uint32_t)off > (uint32_t)(op + ll);
                // (the output bound per step too: op and lp are 32-bit, and up to 2^15 sequences of < 2^18 bytes
                // each could wrap op back into range before the block-end check; such a frame goes to the one-wave
                // decoder, whose verdict is ZSTD_execSequence's.  With it op <= n at every step, so lp <= op never
                // wraps either.)
                const bool lim17 = ((ll | ml) >= (1 << kLenBits)) | (op + ll + ml > n);
                r0 = (uint32_t)ll | ((uint32_t)ml << kLenBits);
                r1 = ((uint32_t)ml >> (32 - kLenBits)) | ((uint32_t)off << (2 * kLenBits - 32));
                keep = !(bad | lim17);
                lp += ll;
                op += ll + ml;
                i++;
                if (bad | lim17 | lastq) {   // an error, a limit, or the block's end (its last literals)
                    const int rem = rs - lp;
                    if (bad | lim17) {
                        res = bad ? ZC : kLegacy;
                        phase = 3;
                    } else if ((P < lo) | (P - lo > ns) | (rem < 0) | (rem > n - op)) {
                        res = ZC;
                        phase = 3;
                    } else {
                        op += rem;
                        phase = 0;
                    }
                    lowok = 1 << 30;
                }
                if (LZH_ZSTD_STATS) sst[4]++;
            }
            seqp[sfl] = (uint64_t)r0 | ((uint64_t)r1 << 32);
            sfl += keep;
        }
    }
    if (LZH_ZSTD_STATS && stats && lane == 0) {
        for (int k = 0; k < 6; k++) atomicAdd(&stats[k], (unsigned long long)sst[k]);
        atomicAdd(&stats[8], (unsigned long long)(__builtin_amdgcn_s_memtime() - tm0));   // (the in-kernel clock)
        atomicAdd(&stats[9], (unsigned long long)(__builtin_amdgcn_s_memrealtime() - tr0));
    }
    if (LZH_ZSTD_STATS && stats && live && res == kLegacy) atomicAdd(&stats[6], 1ull);
    if (live) zfr[f].sv = res;   // (kGo, kLegacy or an error: lzh_zstd_exec_kernel applies it)
}

namespace zsplit {

// one frame's output from its blocks and sequences (one wave)
__device__ __forceinline__ int exec_frame(const Bytes& rin, const Bytes& rout, const Bytes& lout, ZSink& O, LDSA uint8_t* mark,
                                          const uint8_t* zb, const ZLayout& Z, const ZFrame& fr, int lane) {
    const ZBlk* blk = (const ZBlk*)zb;
    const ZExe* ex = (const ZExe*)(zb + Z.exe());
    const uint64_t* seqs = (const uint64_t*)(zb + Z.seqs());
    ZWin fw, lw;
    fw.bind(rin, nullptr);
    int op = 0;
    for (int b = 0; b < fr.nblk; b++) {
        const uint32_t type = blk[b].type, pos = blk[b].pos, size = blk[b].size;
        if (type == 0) {
            fw.load((int)pos, lane);
            O.literals(fw, rin, (int)pos, op, (int)size, lane);
            op += (int)size;
            continue;
        }
        if (type == 1) {
            for (int base = 0; base < (int)size; base += LZH_WAVE) {
                if (base + lane < (int)size) O.put(op + base + lane, pos);
                O.maybe_flush(op + min(base + LZH_WAVE, (int)size), lane);
            }
            op += (int)size;
            continue;
        }
        const Bytes& lsrc = blk[b].ltype == 0 ? rin : lout;
        const int lpos = (int)blk[b].lit, rs = (int)blk[b].rs, nseq = (int)blk[b].nseq;
        const uint64_t* S = seqs + ex[b].seq0;
        lw.bind(lsrc, nullptr);
        lw.load(lpos, lane);
        int lp = 0;
        for (int s0 = 0; s0 < nseq;) {
            const int i = s0 + lane;
            const bool v = i < nseq;
            const uint64_t q = v ? S[i] : 0ull;
            const int ll = (int)(q & ((1u << kLenBits) - 1u)), ml = (int)((q >> kLenBits) & ((1u << kLenBits) - 1u));
            const int off = (int)(q >> (2 * kLenBits));
            const bool big = ll > 255 || ml > 4095;
            const int lin = groups::wave_incl_scan(ll);
            const int k = ffs64(ballot(!v || big || lin > 384));
            if (k > 0) {   // the first k sequences as a group
                const int o = ll + ml;
                const int oin = groups::wave_incl_scan(o);
                const int gl = rdlanei(lin, k - 1), go = rdlanei(oin, k - 1);
                const int ip = lpos + lp;
                if (!lw.covers(ip, ip + gl + 16)) lw.load(ip, lane);
                const uint64_t keep = k == LZH_WAVE ? ~0ull : ((1ull << k) - 1ull);
                groups::emit_group(lw, O, mark, ip, op, go, keep, oin - o, (uint32_t)ll | ((uint32_t)ml << 16),
                                   (uint32_t)(lin - ll), off, lane);
                op += go;
                lp += gl;
                s0 += k;
            } else {       // a long sequence on its own
                const int bl = rdlanei(ll, 0), bm = rdlanei(ml, 0), bo = rdlanei(off, 0);
                O.literals(lw, lsrc, lpos + lp, op, bl, lane);
                O.match(op + bl, bo, bm, lane);
                op += bl + bm;
                lp += bl;
                s0 += 1;
            }
        }
        const int rem = rs - lp;
        if (rem > 0) {
            O.literals(lw, lsrc, lpos + lp, op, rem, lane);
            op += rem;
        }
    }
    O.flush(op, lane);
    if (fr.ccrc >= 0) {   // ZSTD_decompressFrame's checksum check (zstd_decompress.c:1011-1020)
        wait_vm();
        fw.load(fr.ccrc, lane);
        const uint32_t want = fword(fw, fr.ccrc, lane);
        if ((uint32_t)xxh64_wave(O.out, op, lane) != want) return kErrChecksum;
    }
    return op;
}

}  // namespace zsplit

extern "C" __global__ void __launch_bounds__(64)
lzh_zstd_hdr_kernel(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets, const uint32_t* csizes,
                    uint64_t n_total, uint64_t chunk_size, uint8_t* out, int32_t* status, uint8_t* zt, int32_t* zst,
                    zsplit::ZFrame* zfr, unsigned long long* stats, zsplit::ZHuf* jobs, uint32_t* njobs) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_raw[(zstdd::kLdsHdr + 3) / 4];
    LDSA zstdd::Lds& L = *(LDSA zstdd::Lds*)lds_raw;
    const int lane = threadIdx.x;
    const uint64_t chunk = blockIdx.x;
    const uint64_t ooff = chunk * chunk_size;
    if (ooff >= n_total) return;
    const int part = (int)min(chunk_size, n_total - ooff);
    const uint64_t ioff = offsets[chunk];
    const int cs = (int)csizes[chunk];
    const uint64_t readable = ioff < packed_readable ? min<uint64_t>(packed_readable - ioff, (uint64_t)cs + 16) : 0;
    Bytes rin, rout;
    rin.init(packed + ioff, readable);
    rout.init(out + ooff, (uint64_t)part);
    if (cs == part) {                                  // stored raw by the chunk loop (lzbench.cpp:284-288)
        copy_raw(rin, rout, part, lane);
        if (lane == 0) {
            status[chunk] = part;
            zst[chunk] = zsplit::kDone;
        }
        return;
    }
    const zsplit::ZLayout Z = zsplit::zlayout(chunk_size);
    zsplit::ZFrame fr{0, 0, -1, 0, 0, 0, 0, 0};
    const int r = zsplit::hdr_frame(rin, rout, cs, L, part, zt + chunk * Z.stride, Z, fr, lane, stats, jobs, njobs,
                                    (uint32_t)chunk);
    if (lane == 0) {
        if (r == zsplit::kGo) zfr[chunk] = fr;
        zst[chunk] = r == zsplit::kGo ? zsplit::kGo : (r == zsplit::kLegacy ? zsplit::kLegacy : zsplit::kDone);
        if (r < 0) status[chunk] = r;
    }
}

// Huffman literal streams, one stream per lane: 4 sections a wave (lanes 4q + j: section q, stream
// j), 8 waves per CU.  LDS: the sections' tables (2^11 cells each, rows of 16 lanes x 4 bytes as an
// LDS-DMA writes them: section q's dword d at row d / 4, lane 4q + d mod 4), the streams' bit rings
// (32 rows: stream dword d at row d mod 32, two halves of 16-dword blocks, + a mirror of row 0), the
// decoded bytes staged between flush points.  One symbol per lane per step (HUF_decodeSymbolX1: a
// tl-bit lookup, bits below the stream start read as zero); uniform points every kHB steps as in the
// sequence kernel.  A stream not consumed exactly (huf_streams' verdict 1) sends its frame to the
// one-wave decoder when the reference would use the double-symbol decoder there, else it is corrupt.
namespace zsplit {
constexpr int kHB = 16;                          // steps between uniform points (= bytes staged per lane)
// streams lzh_zstd_hufpar_kernel decodes a wave each (the rest: a lane each here)
constexpr int kParMin = 4096;                   // symbols (>= 64 bits a share)
// stream bytes staged in LDS (37 KiB a wave with the table: 4 waves per CU; a 4-stream section of 128 KiB of
// literals has streams of 32 K symbols under 8 bits each, or its literals would not be Huffman-coded)
constexpr int kParCap = 32 * 1024;
__host__ __device__ inline bool huf_par(int on, int nsym, uint32_t sz) {
    return on && nsym >= kParMin && sz + 8 <= (uint32_t)kParCap;
}
}  // namespace zsplit

// HJ sections a wave (4 HJ lanes in use).  The kernel is bound by instruction issue, not by its LDS round
// trips: 8 sections a wave (36 KiB of LDS, one wave per SIMD) issue half the instructions per section of
// 4 a wave (two waves per SIMD) -- 1 GiB -b128: mixed 5.3 -> 4.9 ms, text 2.0 -> 1.6 ms; 2 a wave 6.5 /
// 3.2 ms -- but need 32 sections per CU to keep every SIMD busy, so launches with fewer frames keep 4.
template <int HJ>
__device__ __forceinline__ void zstd_huf(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                                         uint64_t n_total, uint64_t chunk_size, uint8_t* out, int32_t* status,
                                         uint8_t* zt, int32_t* zst, const zsplit::ZHuf* jobs, const uint32_t* njobs,
                                         unsigned long long* stats, int par) {
    using namespace zsplit;
    using namespace zstdd;
    constexpr int kHJ = HJ, kHL = 4 * kHJ;          // sections a wave, lanes in use
    constexpr int kHRow = 4 * kHL;                   // bytes per LDS row (one dword per lane in use)
    constexpr int kHLdsRing = 256 * kHRow, kHLds = kHLdsRing + 33 * kHRow;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kHLds];
    LDSA uint8_t* const S = (LDSA uint8_t*)lds;
    const int lane = threadIdx.x;
    const int q = lane >> 2, j = lane & 3;
    const uint32_t jid = blockIdx.x * kHJ + (uint32_t)q;
    const bool jlive = lane < kHL && jid < *njobs;
    uint32_t jf = 0, jtblk = 0, jtl = 0, jx2 = 0, jns = 0, jdst = 0, jseg = 0, jlast = 0, js0 = 0, jsz = 0;
    if (jlive) {
        const ZHuf* J = jobs + jid;
        jf = J->frame; jtblk = J->tblk; jtl = J->tl; jx2 = J->x2; jns = J->ns; jdst = J->dst; jseg = J->seg;
        jlast = J->last; js0 = J->s0[j]; jsz = J->sz[j];
    }
    bool slive = jlive && zst[jf] == kGo && (uint32_t)j < jns &&
                 !huf_par(par, j == 3 ? (int)jlast : (int)jseg, jsz);   // (long streams: lzh_zstd_hufpar_kernel)
    const ZLayout Z = zlayout(chunk_size);
    // resources from the wave's lowest frame: the packed streams and the table slots (per-lane 32-bit
    // offsets; a section whose offsets would not fit goes to the one-wave decoder)
    uint32_t fmin = jlive ? jf : 0xffffffffu;
    for (int k = 1; k < 64; k <<= 1) fmin = min(fmin, (uint32_t)__shfl_xor((int)fmin, k));
    fmin = uni(fmin == 0xffffffffu ? 0u : fmin);
    const int64_t readable = (int64_t)packed_readable;
    const uint8_t* zb0 = zt + (uint64_t)fmin * Z.stride;
    const rsrc_t rz = rsrc_over(zb0, (uint64_t)0xffffffffull);
    const uint64_t toff = (uint64_t)(jf - fmin) * Z.stride + Z.hufs() + (uint64_t)jtblk * kHufSlot;
    bool far_ = jlive && toff + kHufSlot > 0xffffffffull;
    const uint64_t nfr = chunk_size ? (n_total + chunk_size - 1) / chunk_size : 0;
    uint8_t* const dummy = zt + nfr * Z.stride + (64ull * blockIdx.x) % zdummy_bytes(nfr);   // (spread like the seq kernel's)
    const int l4 = lane * 4;
    const int tl = (int)jtl;
    // this lane's stream
    int P = 0, lo = 0, nsym = 0, done = 0;
    int64_t A = 0;
    uint8_t* dst = out;
    if (slive) {
        const int64_t s0 = (int64_t)offsets[jf] + (int64_t)js0;
        A = s0 & ~3ll;

        const int x0 = (int)(s0 & 3), X = x0 + (int)jsz - 1;
        lo = 8 * x0;
        P = 8 * X + hb32((uint32_t)packed[A + X]);   // (the end mark: checked non-zero by the header kernel)
        nsym = j == 3 ? (int)jlast : (int)jseg;
        dst = out + (uint64_t)jf * chunk_size + jdst + (uint64_t)j * jseg;
    }
    int hb0 = 0, hb1 = 0, rdy = 0, req = 0, iss = 0;
    {
        const int bt = (P - 1) >> 9;
        hb0 = (bt & 1) ? bt - 1 : bt;
        hb1 = (bt & 1) ? bt : bt - 1;
        req = slive ? 3 : 0;
    }
    {   // (a section whose offsets do not fit: its frame goes to the one-wave decoder)
        const uint64_t fm = ballot(far_);
        if (fm) {
            const bool qfar = ((fm >> (4 * q)) & 15ull) != 0;
            if (qfar && j == 0 && jlive) atomicMax(&zst[jf], kLegacy);
            slive = slive && !qfar;
        }
    }
    int res = 0;                                  // 0 going, 1 exact, 2 not exact
    auto fld = [&](int bq, int w) -> uint32_t {
        const LDSA uint8_t* a = S + kHLdsRing + ((bq >> 5) & 31) * kHRow + l4;
        const uint32_t v = __builtin_amdgcn_alignbit(*(const LDSA uint32_t*)(a + kHRow), *(const LDSA uint32_t*)a,
                                                     (uint32_t)bq & 31u);
        return __builtin_amdgcn_ubfe(v, 0u, (uint32_t)w);
    };
    if (!slive) req = 0;
    bool going = slive;
    int lowok = 1 << 30;                         // a step runs while P >= lowok (the ready blocks + tl bits)
    uint64_t hst[5] = {0, 0, 0, 0, 0}, tmark = 0;   // (LZH_ZSTD_STATS: points, steps, intervals, waits, symbols)
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
    for (int ival = 0;; ival++) {
        if (LZH_ZSTD_STATS) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            if (ival) hst[1] += t - tmark;
            tmark = t;
            hst[2]++;
        }
        // ---- uniform point: every memory operation but the last interval's kHB byte stores is done
        __builtin_amdgcn_s_waitcnt(vmcnt_imm(kHB));
        if (LZH_ZSTD_STATS) hst[3] += __builtin_amdgcn_s_memtime() - tmark;
        rdy |= iss;
        iss = 0;
        if (going && done == nsym) {             // huf_streams' verdict: exactly consumed
            res = P == lo ? 1 : 2;
            going = false;
        }
        if (going) {   // the upper block, once the reader is below it, takes the block under the lower one
            const int top = (P - 1) >> 9;
            if ((rdy & 1) && hb0 > top && hb0 > hb1) { hb0 = hb1 - 1; rdy &= ~1; req |= 1; }
            if ((rdy & 2) && hb1 > top && hb1 > hb0) { hb1 = hb0 - 1; rdy &= ~2; req |= 2; }
        }
        if (ival == 0 && ballot(jlive)) {   // the sections' tables: row r = dwords 4r .. 4r+3
            if (jlive) {
                const uint32_t o = (uint32_t)toff + 4 * j;
#pragma unroll 1
                for (int r = 0; r < 256; r += 16) {
                    LDSA uint8_t* d = S + r * kHRow;
                    const uint32_t orr = o + 16 * r;
                    dma_rs(rz, d, orr); dma_rs(rz, d + kHRow, orr + 16); dma_rs(rz, d + 2 * kHRow, orr + 32);
                    dma_rs(rz, d + 3 * kHRow, orr + 48); dma_rs(rz, d + 4 * kHRow, orr + 64);
                    dma_rs(rz, d + 5 * kHRow, orr + 80); dma_rs(rz, d + 6 * kHRow, orr + 96);
                    dma_rs(rz, d + 7 * kHRow, orr + 112); dma_rs(rz, d + 8 * kHRow, orr + 128);
                    dma_rs(rz, d + 9 * kHRow, orr + 144); dma_rs(rz, d + 10 * kHRow, orr + 160);
                    dma_rs(rz, d + 11 * kHRow, orr + 176); dma_rs(rz, d + 12 * kHRow, orr + 192);
                    dma_rs(rz, d + 13 * kHRow, orr + 208); dma_rs(rz, d + 14 * kHRow, orr + 224);
                    dma_rs(rz, d + 15 * kHRow, orr + 240);
                }
            }
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if (ballot(req & (1 << h))) {   // the block's 16 dwords (global_load_lds rows: see the sequence kernel)
                const int64_t x0 = A + 64ll * (h ? hb1 : hb0);
                // a block wholly outside the packed bytes holds no stream data: any readable bytes will do
                const bool part = x0 >= 0 && x0 < readable && x0 + 64 > readable;
                const uint8_t* g = packed + (x0 < 0 || x0 >= readable ? 0 : x0);
                LDSA uint8_t* d = S + kHLdsRing + h * 16 * kHRow;
                if ((req & (1 << h)) && !part) {
#pragma unroll
                    for (int k = 0; k < 16; k++) dma_row(g + 4 * k, d + k * kHRow);
                    if (h == 0) dma_row(g, S + kHLdsRing + 32 * kHRow);   // (the mirror of row 0)
                }
                if (ballot((req & (1 << h)) && part)) {   // (the packed bytes end inside the block)
                    if ((req & (1 << h)) && part) {
                        for (int k = 0; k < 16; k++)
                            dma_row(packed + (x0 + 4 * k < readable - 4 ? x0 + 4 * k : ((readable - 4) & ~3ll)), d + k * kHRow);
                        if (h == 0) dma_row(packed + x0, S + kHLdsRing + 32 * kHRow);
                    }
                }
                if (req & (1 << h)) {
                    req &= ~(1 << h);
                    iss |= 1 << h;
                }
            }
        }
        lowok = (rdy == 3 ? 512 * min(hb0, hb1) : (rdy == 1 ? 512 * hb0 : (rdy == 2 ? 512 * hb1 : (1 << 30)))) + 12;
        if (!going) lowok = 1 << 30;
        if (LZH_ZSTD_STATS) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            hst[0] += t - tmark;
            tmark = t;
        }
        if (!ballot(going)) break;
        if (ival > 2 * kBlockMax) {   // (a bound every stream meets)
            if (going) { going = false; res = 2; }
            lowok = 1 << 30;
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- kHB steps, one symbol each (HUF_decodeSymbolX1) and exactly one byte store per lane (a dummy
        // byte for a lane without a symbol), so that the next point's vmcnt(kHB) waits for the fills only
#pragma unroll 2
        for (int k = 0; k < kHB; k++) {
            const bool act = P >= lowok && done < nsym;
            const int bq = P - tl;
            uint32_t v = fld(bq, tl);
            if (bq < lo) v &= lo - bq >= 32 ? 0u : (~0u << (lo - bq));   // (zero-padded below the start)
            const uint32_t e = *(const LDSA uint16_t*)(S + (v >> 3) * kHRow + (q << 4) + (v & 7) * 2);
            *(act ? dst + done : dummy + lane) = (uint8_t)e;
            P -= act ? (int)(e >> 8) : 0;
            done += act;
        }
    }
    if (LZH_ZSTD_STATS && stats && lane == 0) {
        for (int k = 0; k < 4; k++) atomicAdd(&stats[k], (unsigned long long)hst[k]);
    }
    if (LZH_ZSTD_STATS && stats && slive) atomicAdd(&stats[4], (unsigned long long)nsym);
    if (LZH_ZSTD_STATS && stats && slive && res == 2) atomicAdd(&stats[5 + (int)jx2], 1ull);
    if (LZH_ZSTD_STATS && stats && far_) atomicAdd(&stats[7], 1ull);
    if (slive && res == 2) {   // not consumed exactly: X2's verdict (the one-wave decoder) or corrupt
        if (jx2) {
            atomicMax(&zst[jf], kLegacy);
        } else if (atomicMax(&zst[jf], kDone) != kDone) {
            status[jf] = ZC;
        }
    }
}

// Long Huffman streams, one per WAVE (self-synchronising parallel decode).  A 4-stream literal section of a
// frame with few matches holds up to 32 K symbols a stream, and one lane's serial decode of it -- two
// dependent LDS round trips a symbol -- bounds lzh_zstd_huf_kernel (config 5's 512 MiB share: a third of
// the frames are whole-block literals).  Here the stream's bits are cut into 64 equal shares, one per lane:
// every lane decodes its share from its top (lane 0 from the stream's start, the others from a guess),
// recording where its chain leaves the share and how many symbols it took; a lane whose true start -- the
// previous lane's exit -- differs from the one it used decodes again from there (Huffman codes
// resynchronise within a few symbols, so after one such round the exits no longer move); the symbol
// counts' prefix sum places every share's output, and a last pass writes it.  The chain from the stream's
// start is the serial decoder's, so the verdict is huf_streams': exact iff it ends exactly at the start of
// the stream's bits after exactly nsym symbols (else the frame goes to the one-wave decoder (X2) or is
// corrupt, as in lzh_zstd_huf_kernel).

extern "C" __global__ void __launch_bounds__(64)
lzh_zstd_hufpar_kernel(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets, uint64_t chunk_size,
                       uint8_t* out, int32_t* status, uint8_t* zt, int32_t* zst, const zsplit::ZHuf* jobs,
                       const uint32_t* njobs, int par) {
    using namespace zsplit;
    using namespace zstdd;
    __shared__ __attribute__((aligned(16))) uint32_t sbuf[kParCap / 4 + 128];   // dword d of the stream at d + 1
    __shared__ __attribute__((aligned(16))) uint16_t tab[2048];
    const int lane = threadIdx.x;
    const uint32_t jid = blockIdx.x >> 2, j = blockIdx.x & 3u;
    if (jid >= *njobs) return;
    const ZHuf* J = jobs + jid;
    const uint32_t jf = uni(J->frame), jns = uni(J->ns), jseg = uni(J->seg), jlast = uni(J->last);
    if (j >= jns) return;
    const int nsym = (int)(j == 3 ? jlast : jseg);
    const uint32_t sz = uni(J->sz[j]);
    if (!huf_par(par, nsym, sz) || uni((uint32_t)zst[jf]) != (uint32_t)kGo) return;
    const ZLayout Z = zlayout(chunk_size);
    const int tl = (int)uni(J->tl);
    {   // the section's table (2^11 16-bit cells: symbol | nbBits << 8)
        const uint32_t* tb = (const uint32_t*)(zt + (uint64_t)jf * Z.stride + Z.hufs() + (uint64_t)uni(J->tblk) * kHufSlot);
        for (int i = lane; i < 1024; i += LZH_WAVE) ((LDSA uint32_t*)tab)[i] = tb[i];
    }
    // the stream's bytes [A, A + X] (A 4-aligned, the stream starting at byte x0), bits below its start zero
    const int64_t s0 = (int64_t)offsets[jf] + (int64_t)uni(J->s0[j]);
    const int64_t A = s0 & ~3ll;
    const int x0 = (int)(s0 & 3), X = x0 + (int)sz - 1;
    const int lo = 8 * x0;
    const int nd = (X + 4) >> 2;
    const int64_t avail = (int64_t)packed_readable - A;
    const rsrc_t r = make_rsrc(packed + A, (uint32_t)max<int64_t>(0, min<int64_t>(avail, (int64_t)nd * 4)));
    {
        if (lane == 0) sbuf[0] = 0u;
        // (LDS-DMA rows of 64 dwords, one wait; past nd the range check reads zeros)
        for (int d0 = 0; d0 < nd + 2; d0 += LZH_WAVE)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(sbuf + 1 + d0), 4,
                                                     4 * (d0 + lane), 0, 0, 0);
    }
    wait_vm();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): table and stream in LDS
    const uint32_t lastb = (sbuf[(X >> 2) + 1] >> (8 * (X & 3))) & 0xffu;
    // bits [bq, bq + tl) (bq >= -32: the zero dword below the stream), zero below lo
    auto bits = [&](int bq) -> uint32_t {
        const int b = bq + 32, d = b >> 5;
        const volatile LDSA uint32_t* s = (const volatile LDSA uint32_t*)sbuf;
        uint32_t v = __builtin_amdgcn_ubfe(__builtin_amdgcn_alignbit(s[d + 1], s[d], (uint32_t)b & 31u), 0u, (uint32_t)tl);
        if (bq < lo) v &= lo - bq >= 32 ? 0u : (~0u << (lo - bq));
        return v;
    };
    const int P0 = 8 * X + (lastb ? hb32(lastb) : 0);   // (the end mark: checked non-zero by the header kernel)
    // this lane's share (P0 - lane * seg, P0 - (lane + 1) * seg], the last one down to lo
    const int nbits = P0 - lo;
    const int seg = (nbits + LZH_WAVE - 1) / LZH_WAVE;
    const int top = P0 - lane * seg;
    const int bot = lane == LZH_WAVE - 1 ? lo : max(P0 - (lane + 1) * seg, lo);
    const int guard = seg + 64;
    // decode the share from start: the chain's exit (the first symbol top at or below bot) and its symbols
    auto pass = [&](bool act, int start, int& ex, int& cnt, uint8_t* wdst) {
        int P = start, c = 0;
        for (int it = 0; it < guard; it++) {
            const bool go = act && P > bot;
            if (!ballot(go)) break;
            if (go) {
                const uint32_t e = ((const volatile LDSA uint16_t*)tab)[bits(P - tl)];
                if (wdst) wdst[c] = (uint8_t)e;
                P -= (int)(e >> 8);
                c++;
            }
        }
        if (act) { ex = P; cnt = c; }
    };
    int start = lane == 0 ? P0 : top, ex = 0, cnt = 0;
    pass(true, start, ex, cnt, nullptr);
    for (int round = 0; round < LZH_WAVE; round++) {   // until every share starts where the previous one ends
        const int prev = (int)lane_gather((uint32_t)ex, lane > 0 ? lane - 1 : 0);
        const int want = lane == 0 ? P0 : prev;
        const bool ch = want != start;
        if (!ballot(ch)) break;
        // decode from the new start (A) alongside the chain already counted from the old one (B), always the
        // higher of the two, until they meet -- the rest is the counted chain -- or A leaves the share
        int PA = want, cA = 0, PB = start, cB = 0;
        bool met = false;
        for (int it = 0; it < 2 * guard; it++) {
            met = met || (ch && PA == PB);
            const bool go = ch && !met && PA > bot;
            if (!ballot(go)) break;
            if (go) {
                const bool a = PA > PB;
                const uint32_t e = ((const volatile LDSA uint16_t*)tab)[bits((a ? PA : PB) - tl)];
                const int nb = (int)(e >> 8);
                PA -= a ? nb : 0;
                cA += a ? 1 : 0;
                PB -= a ? 0 : nb;
                cB += a ? 0 : 1;
            }
        }
        if (ch) {
            if (met) {
                cnt = cA + (cnt - cB);   // (ex: the counted chain's exit)
            } else {
                ex = PA;
                cnt = cA;
            }
            start = want;
        }
    }
    const int incl = groups::wave_incl_scan(cnt);
    const int total = rdlanei(incl, LZH_WAVE - 1);
    const bool exact = total == nsym && rdlanei(ex, LZH_WAVE - 1) == lo;
    if (exact) {
        uint8_t* dst = out + (uint64_t)jf * chunk_size + uni(J->dst) + (uint64_t)j * jseg + (incl - cnt);
        int ex2 = 0, cnt2 = 0;
        pass(true, start, ex2, cnt2, dst);
    } else if (lane == 0) {   // not consumed exactly: X2's verdict (the one-wave decoder) or corrupt
        if (uni(J->x2)) {
            atomicMax(&zst[jf], kLegacy);
        } else if (atomicMax(&zst[jf], kDone) != kDone) {
            status[jf] = ZC;
        }
    }
}

extern "C" __global__ void __launch_bounds__(64)
lzh_zstd_huf_kernel(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets, uint64_t n_total,
                    uint64_t chunk_size, uint8_t* out, int32_t* status, uint8_t* zt, int32_t* zst,
                    const zsplit::ZHuf* jobs, const uint32_t* njobs, unsigned long long* stats, int par) {
    zstd_huf<4>(packed, packed_readable, offsets, n_total, chunk_size, out, status, zt, zst, jobs, njobs, stats, par);
}
extern "C" __global__ void __launch_bounds__(64)
lzh_zstd_huf8_kernel(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets, uint64_t n_total,
                     uint64_t chunk_size, uint8_t* out, int32_t* status, uint8_t* zt, int32_t* zst,
                     const zsplit::ZHuf* jobs, const uint32_t* njobs, unsigned long long* stats, int par) {
    zstd_huf<8>(packed, packed_readable, offsets, n_total, chunk_size, out, status, zt, zst, jobs, njobs, stats, par);
}

// The sequence / execution plan: frames the header and literal kernels left at kGo, split by their sequence
// count -- long (nsq > max / 2) at the back of `flist`, short at the front, each in frame order -- so that the
// execution of the short frames runs while the long ones still decode (the sequence kernel's time is its
// longest chains').  One workgroup of 1024 threads; fcnt = {short, long}.
extern "C" __global__ void __launch_bounds__(1024)
lzh_zstd_plan_kernel(const int32_t* zst, const zsplit::ZFrame* zfr, uint32_t nchunks, uint32_t* flist, uint32_t* fcnt) {
    __shared__ uint32_t smax, wsum[2][16], base[2];
    const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
    if (t == 0) { smax = 0; base[0] = 0; base[1] = 0; }
    __syncthreads();
    uint32_t m = 0;
    for (uint32_t i = t; i < nchunks; i += 1024)
        if (zst[i] == zsplit::kGo) m = max(m, (uint32_t)max(zfr[i].nsq, 0));
    atomicMax(&smax, m);
    __syncthreads();
    const uint32_t thr = smax / 2;
    for (uint32_t i0 = 0; i0 < nchunks; i0 += 1024) {
        const uint32_t i = i0 + t;
        const bool go = i < nchunks && zst[i] == zsplit::kGo;
        const bool lng = go && (uint32_t)max(zfr[i].nsq, 0) > thr;
        const uint64_t bs = __builtin_amdgcn_ballot_w64(go && !lng), bl = __builtin_amdgcn_ballot_w64(lng);
        const uint64_t below = (1ull << lane) - 1ull;
        if (lane == 0) { wsum[0][w] = (uint32_t)__builtin_popcountll(bs); wsum[1][w] = (uint32_t)__builtin_popcountll(bl); }
        __syncthreads();
        uint32_t ps = base[0], pl = base[1];
        for (uint32_t k = 0; k < w; k++) { ps += wsum[0][k]; pl += wsum[1][k]; }
        if (go && !lng) flist[ps + (uint32_t)__builtin_popcountll(bs & below)] = i;
        if (lng) flist[nchunks - 1 - (pl + (uint32_t)__builtin_popcountll(bl & below))] = i;
        __syncthreads();
        if (t == 0)
            for (uint32_t k = 0; k < 16; k++) { base[0] += wsum[0][k]; base[1] += wsum[1][k]; }
        __syncthreads();
    }
    if (t == 0) {
        // the long list rounded up to whole sequence waves with the short list's last frames, so that the two
        // launches' frames need no more waves than one launch's (a wave more than there are SIMDs would wait
        // for a whole chain); the ranges are disjoint or the entries already in place (see the indices)
        uint32_t ns = base[0], nl = base[1];
        const uint32_t m = min((uint32_t)(zsplit::kFPW - nl % zsplit::kFPW) % zsplit::kFPW, ns);
        for (uint32_t j = 0; j < m; j++) flist[nchunks - 1 - (nl + j)] = flist[ns - 1 - j];
        fcnt[0] = ns - m;
        fcnt[1] = nl + m;
    }
}

extern "C" __global__ void __launch_bounds__(64)
lzh_zstd_exec_kernel(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets, const uint32_t* csizes,
                     uint64_t n_total, uint64_t chunk_size, uint8_t* out, int32_t* status, const uint8_t* zt,
                     int32_t* zst, const zsplit::ZFrame* zfr, const uint32_t* flist, const uint32_t* fcnt, int which,
                     uint32_t nchunks) {
    __shared__ __attribute__((aligned(16))) uint8_t win[zstdd::kZW + 3 * LZH_WAVE];
    const int lane = threadIdx.x;
    if (which >= 0 && blockIdx.x >= fcnt[which]) return;
    const uint64_t chunk = which < 0 ? blockIdx.x : (which == 0 ? flist[blockIdx.x] : flist[nchunks - 1 - blockIdx.x]);
    const uint64_t ooff = chunk * chunk_size;
    if (ooff >= n_total || zst[chunk] != zsplit::kGo) return;   // (the header / literal kernels' verdict first)
    const int sv = zfr[chunk].sv;                                // then the sequence kernel's
    if (sv != zsplit::kGo) {
        if (lane == 0) {
            if (sv == zsplit::kLegacy) {
                zst[chunk] = zsplit::kLegacy;
            } else {
                status[chunk] = sv;
                zst[chunk] = zsplit::kDone;
            }
        }
        return;
    }
    const int part = (int)min(chunk_size, n_total - ooff);
    const uint64_t ioff = offsets[chunk];
    const int cs = (int)csizes[chunk];
    const uint64_t readable = ioff < packed_readable ? min<uint64_t>(packed_readable - ioff, (uint64_t)cs + 16) : 0;
    Bytes rin, rout, lout;
    rin.init(packed + ioff, readable);
    rout.init(out + ooff, (uint64_t)part);
    lout.init(out + ooff, (uint64_t)part + 3);
    const zsplit::ZLayout Z = zsplit::zlayout(chunk_size);
    zstdd::ZSink O{(LDSA uint8_t*)win, rout, 0, 0};
    const int r = zsplit::exec_frame(rin, rout, lout, O, (LDSA uint8_t*)win + zstdd::kZW, zt + chunk * Z.stride, Z,
                                     zfr[chunk], lane);
    if (lane == 0) status[chunk] = r;
}

#ifndef LZH_ZSTD_MINW
#define LZH_ZSTD_MINW 1   // waves per SIMD the register allocation must allow (LDS allows 3)
#endif
extern "C" __global__ void __launch_bounds__(64, LZH_ZSTD_MINW)
lzh_zstd_decompress_kernel(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                           const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint8_t* out,
                           int32_t* status, uint32_t chunk0, unsigned long long* stats, const int32_t* zsel) {
    __shared__ __attribute__((aligned(16))) uint32_t lds_raw[(sizeof(zstdd::Lds) + 3) / 4];
    LDSA zstdd::Lds& L = *(LDSA zstdd::Lds*)lds_raw;
    const int lane = threadIdx.x;
    const uint64_t chunk = (uint64_t)blockIdx.x + chunk0;
    const uint64_t ooff = chunk * chunk_size;
    if (ooff >= n_total) return;
    if (zsel && zsel[chunk] != zsplit::kLegacy) return;   // (decoded by the split kernels)
    const int part = (int)min(chunk_size, n_total - ooff);
    const uint64_t ioff = offsets[chunk];
    const int cs = (int)csizes[chunk];
    // (+16: whole-dword reads of the frame's last bytes; bytes past the frame are never used)
    const uint64_t readable = ioff < packed_readable ? min<uint64_t>(packed_readable - ioff, (uint64_t)cs + 16) : 0;
    Bytes rin, rout;
    rin.init(packed + ioff, readable);
    rout.init(out + ooff, (uint64_t)part);
    int r;
    if (cs == part) {                                  // stored raw by the chunk loop (lzbench.cpp:284-288)
        copy_raw(rin, rout, part, lane);
        r = part;
    } else {
        zstdd::ZSink O{(LDSA uint8_t*)L.win, rout, 0, 0};
        for (int i = lane; i < 36 + 53; i += LZH_WAVE) L.base[i] = i < 36 ? zstdd::kLLBase[i] : zstdd::kMLBase[i - 36];
        wave_lds_fence();
        Bytes lout;
        lout.init(out + ooff, (uint64_t)part + 3);
        r = zstdd::decode_frame(rin, lout, cs, O, L, part, lane, stats);
        if (r > 0) O.flush(r, lane);
    }
    if (lane == 0) status[chunk] = r;
}

#include "launch.h"

#include <mutex>
// Test hook: force the LZ4 / snappy decoder's output window (4096, 8192 or 16384; 0 = by chunk count)
// so that the parity tests run every window kernel on the same streams.
static int g_force_window = 0;
// Test hook: 1 = decode zstd frames with the one-wave-per-frame kernel only (no split kernels)
static int g_zstd_legacy = 0;
extern "C" int lzh_debug_zstd_legacy(int on) {
    g_zstd_legacy = on ? 1 : 0;
    return 0;
}
// Test hook: force the zstd literal kernel's sections per wave (4 or 8; 0 = by frame count)
// Test hook: long Huffman streams one per wave (lzh_zstd_hufpar_kernel) on / off
// the sequence kernel on a per-device side stream beside the literal kernels (0: all on the caller's stream)
static int g_zstd_side = 1;
extern "C" int lzh_debug_zstd_side(int on) {
    g_zstd_side = on ? 1 : 0;
    return 0;
}
// Side streams per caller stream (and per slot k): independent callers -- the batched rows' two alternating
// kernel streams, other threads' streams -- never queue behind each other's forked kernels.  Each entry owns its
// fork / join events (a call records and waits them on its own caller stream, in order).  A caller stream on a
// device other than the current one, or past kMaxSide entries, gets no side stream: the caller then launches
// everything on its own stream, in order.
struct SideEntry {
    hipStream_t caller;
    int dev, k;
    hipStream_t ss;
    hipEvent_t fork, join;
};
static constexpr int kMaxSide = 256;
static SideEntry g_side[kMaxSide];
static int g_nside = 0;
static std::mutex g_side_mu;
bool lzh_side_stream(hipStream_t s, hipStream_t& ss, hipEvent_t& fork, hipEvent_t& join, int k) {
    if (k < 0 || k > 1) return false;
    int dev = -1, sdev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return false;
    hipDevice_t d = 0;
    if (hipStreamGetDevice(s, &d) != hipSuccess) return false;
    sdev = (int)d;
    if (sdev != dev) return false;
    std::lock_guard<std::mutex> g(g_side_mu);
    for (int i = 0; i < g_nside; i++)
        if (g_side[i].caller == s && g_side[i].dev == dev && g_side[i].k == k) {
            ss = g_side[i].ss;
            fork = g_side[i].fork;
            join = g_side[i].join;
            return true;
        }
    if (g_nside >= kMaxSide) return false;
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) hi = 0;
    SideEntry e{s, dev, k, nullptr, nullptr, nullptr};
    // (the highest priority: their waves go out before the caller's stream's)
    if (hipStreamCreateWithPriority(&e.ss, hipStreamNonBlocking, hi) != hipSuccess) return false;
    if (hipEventCreateWithFlags(&e.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e.join, hipEventDisableTiming) != hipSuccess) {
        if (e.fork) (void)hipEventDestroy(e.fork);
        (void)hipStreamDestroy(e.ss);
        return false;
    }
    g_side[g_nside++] = e;
    ss = e.ss;
    fork = e.fork;
    join = e.join;
    return true;
}
// (tests: how many side streams the library holds)
extern "C" int lzh_debug_side_streams() {
    std::lock_guard<std::mutex> g(g_side_mu);
    return g_nside;
}
// the sequence / execution plan by sequence count (lzh_zstd_plan_kernel; 0: one sequence launch)
static int g_zstd_plan = 1;
extern "C" int lzh_debug_zstd_plan(int on) {
    g_zstd_plan = on ? 1 : 0;
    return 0;
}
static int g_zstd_hufpar = 1;
extern "C" int lzh_debug_zstd_hufpar(int on) {
    g_zstd_hufpar = on ? 1 : 0;
    return 0;
}
static int g_zstd_huf_sections = 0;
extern "C" int lzh_debug_zstd_huf_sections(int hj) {
    if (hj != 0 && hj != 4 && hj != 8) return -1;
    g_zstd_huf_sections = hj;
    return 0;
}
extern "C" int lzh_debug_force_decode_window(int kw) {
    if (kw != 0 && kw != 4096 && kw != 8192 && kw != 16384) return -1;
    g_force_window = kw;
    return 0;
}

// The LZ4 / snappy decoder's LDS output window for a launch of nchunks on the current device: the
// widest whose occupancy (waves per CU by LDS: 160 KiB in 512-byte granules, at most 32 waves) still
// holds every chunk at once; 4096 = lzh_decompress_v2_kernel, 8192 = _w8k, 16384 = _w16k.
static int decode_window(uint32_t nchunks) {
    if (g_force_window) return g_force_window;
    static int cus[64];
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) dev = 0;
    if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        cus[dev] = 0;
    auto fits = [&](int kw) {
        const int lds = (kw + 3 * LZH_WAVE + kRingBytes + 511) / 512 * 512;
        return (uint64_t)nchunks <= (uint64_t)cus[dev] * (uint64_t)min(32, 160 * 1024 / lds);
    };
    if (LZH_DEC_WIDE && cus[dev] > 0) {
        if (LZH_DEC_WIDE >= 2 && fits(16384)) return 16384;
        if (fits(8192)) return 8192;
    }
    return 4096;
}
// (bench.py names the decode kernel a launch of nchunks runs)
extern "C" int lzh_debug_decode_window(uint32_t nchunks) { return decode_window(nchunks); }

hipError_t lzh_launch_decompress(int codec, const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                                 const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint8_t* out,
                                 int32_t* status, uint32_t nchunks, hipStream_t s, const void* desc) {
    if (nchunks == 0) return hipSuccess;
    const int kw = decode_window(nchunks);
    auto k = kw == 16384 ? lzh_decompress_w16k_kernel : kw == 8192 ? lzh_decompress_w8k_kernel : lzh_decompress_v2_kernel;
    hipLaunchKernelGGL(k, dim3(nchunks), dim3(64), 0, s, codec, packed, packed_readable, offsets, csizes, n_total,
                       chunk_size, out, status, 0u, (const uint32_t*)desc);
    if (desc && codec == 0)   // LZ4 frames: the linked ones (descriptors the kernel above skipped)
        hipLaunchKernelGGL(lzh_decompress_linked_kernel, dim3(nchunks), dim3(64), 0, s, packed, packed_readable, out,
                           status, (const uint32_t*)desc);
    return hipGetLastError();
}

// The split pays where a chunk's serial decode is long against the walk: from 8 fragments (512 KiB)
// (mixed 1 GiB: -b256 walk 3.1 + fragments 3.3 ms against 6.5 ms whole; -b1024 9.2 + 3.4 against 18.5 ms;
// profiles/r05_snsplit).  Test hooks: the mode (0 off: every chunk whole; 1 from kMinFrags fragments;
// 2 from 2 fragments), and the number of chunks finished by fragments (reset with reset != 0).
static int g_snappy_split = 1;
extern "C" int lzh_debug_snappy_split(int mode) {
    if (mode < 0 || mode > 2) return -1;
    g_snappy_split = mode;
    return 0;
}
extern "C" long long lzh_debug_snappy_split_done(int reset) {
    unsigned long long v = 0;
    if (reset) return hipMemcpyToSymbol(HIP_SYMBOL(lzh_snsplit_done), &v, sizeof(v)) == hipSuccess ? 0 : -1;
    if (hipMemcpyFromSymbol(&v, HIP_SYMBOL(lzh_snsplit_done), sizeof(v)) != hipSuccess) return -1;
    return (long long)v;
}

// temp for the fragment-parallel snappy decode (0: chunks of one fragment, or too large to split):
// fragment descriptors (32 B) and statuses, per-chunk split flags and whole-chunk descriptors
size_t lzh_snappy_split_temp(uint64_t n, uint64_t chunk_size) {
    const uint32_t F = snsplit::frags(chunk_size);
    if (!g_snappy_split || F < (g_snappy_split == 2 ? 2u : snsplit::kMinFrags) || F > snsplit::kMaxFrags || n == 0)
        return 0;
    const uint64_t k = (n + chunk_size - 1) / chunk_size;
    auto al = [](uint64_t v) { return (v + 255) & ~(uint64_t)255; };
    return (size_t)(al(k * F * 32) + al(k * F * 4) + al(k * 4) + al(k * 32) + 256);
}

hipError_t lzh_launch_snappy_split_decompress(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                                              const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint8_t* out,
                                              int32_t* status, uint32_t nchunks, uint8_t* temp, hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    const uint32_t F = snsplit::frags(chunk_size);
    const uint64_t k = nchunks;
    auto al = [](uint64_t v) { return (v + 255) & ~(uint64_t)255; };
    uint32_t* desc = (uint32_t*)temp;
    int32_t* fstat = (int32_t*)(temp + al(k * F * 32));
    uint32_t* cflag = (uint32_t*)(temp + al(k * F * 32) + al(k * F * 4));
    uint32_t* sdesc = (uint32_t*)(temp + al(k * F * 32) + al(k * F * 4) + al(k * 4));
    if (k * F > 0xffffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(lzh_snappy_split_kernel, dim3(nchunks), dim3(64), 0, s, packed, packed_readable, offsets, csizes,
                       n_total, chunk_size, F, desc, cflag);
    hipError_t e = lzh_launch_decompress(1, packed, packed_readable, nullptr, nullptr, n_total, chunk_size, out, fstat,
                                         (uint32_t)(k * F), s, desc);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(lzh_snappy_join_kernel, dim3((nchunks + 255) / 256), dim3(256), 0, s, offsets, csizes, n_total,
                       chunk_size, F, desc, fstat, cflag, sdesc, status, nchunks);
    return lzh_launch_decompress(1, packed, packed_readable, nullptr, nullptr, n_total, chunk_size, out, status, nchunks,
                                 s, sdesc);
}

hipError_t lzh_launch_zstd_decompress(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                                      const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint8_t* out,
                                      int32_t* status, uint32_t nchunks, uint8_t* zt, hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    unsigned long long* stats = nullptr;
#if LZH_ZSTD_STATS
    static unsigned long long* d_stats = nullptr;
    if (!d_stats) (void)hipMalloc(&d_stats, zstdd::kZClk * sizeof(unsigned long long));
    (void)hipMemsetAsync(d_stats, 0, zstdd::kZClk * sizeof(unsigned long long), s);
    stats = d_stats;
#endif
    const int32_t* zsel = nullptr;
    if (zt && !g_zstd_legacy) {   // the split kernels; frames they leave go to the one-wave decoder below
        const zsplit::ZLayout Z = zsplit::zlayout(chunk_size);
        int32_t* zst = (int32_t*)(zt + (uint64_t)nchunks * Z.stride + zsplit::zdummy_bytes(nchunks));   // (after the dummy words)
        zsplit::ZFrame* zfr = (zsplit::ZFrame*)((uint8_t*)zst + (((uint64_t)nchunks * 4 + 255) & ~255ull));
        uint32_t* njobs = (uint32_t*)((uint8_t*)zfr + (((uint64_t)nchunks * sizeof(zsplit::ZFrame) + 255) & ~255ull));
        zsplit::ZHuf* jobs = (zsplit::ZHuf*)((uint8_t*)njobs + 256);
        (void)hipMemsetAsync(njobs, 0, 4, s);
        hipLaunchKernelGGL(lzh_zstd_hdr_kernel, dim3(nchunks), dim3(64), 0, s, packed, packed_readable, offsets, csizes,
                           n_total, chunk_size, out, status, zt, zst, zfr, stats, jobs, njobs);
        static int hcus[64];
        int hdev = 0;
        (void)hipGetDevice(&hdev);
        if (hdev < 0 || hdev >= 64) hdev = 0;
        // the sequence kernel needs the header kernel's output only (its verdict goes to zfr[].sv): it runs
        // on a side stream beside the literal kernels, launched first -- its waves, one per SIMD at config 5's
        // share, take their SIMDs and the literal waves fill the rest -- and the execution kernel joins both
        // and after the plan (lzh_zstd_plan_kernel) the frames with the longest sequence chains decode on one
        // side stream, the rest on another, so that the execution kernel runs the short ones while the long
        // ones still decode
        uint32_t* flist = (uint32_t*)((uint8_t*)jobs + (uint64_t)nchunks * Z.bmax * sizeof(zsplit::ZHuf) + 256);
        uint32_t* fcnt = flist + nchunks;
        hipStream_t sq[2] = {s, s};
        hipEvent_t fork[2] = {nullptr, nullptr}, join[2] = {nullptr, nullptr};
        const bool side = !LZH_ZSTD_STATS && g_zstd_side && lzh_side_stream(s, sq[0], fork[0], join[0], 0) &&
                          lzh_side_stream(s, sq[1], fork[1], join[1], 1);
        const unsigned sgrid = (nchunks + zsplit::kFPW - 1) / zsplit::kFPW;
        if (!hcus[hdev] && hipDeviceGetAttribute(&hcus[hdev], hipDeviceAttributeMultiprocessorCount, hdev) != hipSuccess)
            hcus[hdev] = 0;
        // (the plan only while the sequence waves leave LDS room beside them -- at most 2 of a CU's 4 -- for the
        // literal kernels, whose end the execution of the short frames waits for; else one sequence launch)
        const bool plan = side && g_zstd_plan && hcus[hdev] > 0 && sgrid <= 2u * (unsigned)hcus[hdev];
        if (plan) {
            hipLaunchKernelGGL(lzh_zstd_plan_kernel, dim3(1), dim3(1024), 0, s, (const int32_t*)zst,
                               (const zsplit::ZFrame*)zfr, nchunks, flist, fcnt);
            for (int k = 0; k < 2; k++) {   // long list (which 1) on side stream 0, launched first
                (void)hipEventRecord(fork[k], s);
                (void)hipStreamWaitEvent(sq[k], fork[k], 0);
                hipLaunchKernelGGL(lzh_zstd_seq_kernel, dim3(sgrid), dim3(64), 0, sq[k], packed, packed_readable,
                                   offsets, chunk_size, nchunks, status, zt, zst, zfr, nullptr, (const uint32_t*)flist,
                                   (const uint32_t*)fcnt, 1 - k);
                (void)hipEventRecord(join[k], sq[k]);
            }
        } else if (side) {
            (void)hipEventRecord(fork[0], s);
            (void)hipStreamWaitEvent(sq[0], fork[0], 0);
            hipLaunchKernelGGL(lzh_zstd_seq_kernel, dim3(sgrid), dim3(64), 0, sq[0], packed, packed_readable, offsets,
                               chunk_size, nchunks, status, zt, zst, zfr, nullptr, (const uint32_t*)nullptr,
                               (const uint32_t*)nullptr, -1);
            (void)hipEventRecord(join[0], sq[0]);
        }
        const uint64_t maxjobs = (uint64_t)nchunks * Z.bmax;
        unsigned long long* hstats = nullptr;
#if LZH_ZSTD_STATS
        static unsigned long long* d_hst = nullptr;
        if (!d_hst) (void)hipMalloc(&d_hst, 8 * sizeof(unsigned long long));
        (void)hipMemsetAsync(d_hst, 0, 8 * sizeof(unsigned long long), s);
        hstats = d_hst;
#endif
        // (8 sections a wave once the frames -- about one Huffman job each -- fill 8 x 4 waves per CU)
        const int hj = (g_zstd_huf_sections ? g_zstd_huf_sections == 8
                                            : hcus[hdev] > 0 && (uint64_t)nchunks >= 32ull * (uint64_t)hcus[hdev]) ? 8 : 4;
        hipLaunchKernelGGL(hj == 8 ? lzh_zstd_huf8_kernel : lzh_zstd_huf_kernel, dim3((unsigned)((maxjobs + hj - 1) / hj)),
                           dim3(64), 0, s, packed, packed_readable, offsets, n_total, chunk_size, out, status, zt, zst,
                           (const zsplit::ZHuf*)jobs, (const uint32_t*)njobs, hstats, g_zstd_hufpar);
        if (g_zstd_hufpar)   // (off: the per-lane kernel above decoded every stream)
            hipLaunchKernelGGL(lzh_zstd_hufpar_kernel, dim3((unsigned)(maxjobs * 4)), dim3(64), 0, s, packed,
                               packed_readable, offsets, chunk_size, out, status, zt, zst, (const zsplit::ZHuf*)jobs,
                               (const uint32_t*)njobs, g_zstd_hufpar);
#if LZH_ZSTD_STATS
        {
            unsigned long long h[8];
            uint32_t nj = 0;
            (void)hipMemcpyAsync(h, d_hst, sizeof(h), hipMemcpyDeviceToHost, s);
            (void)hipMemcpyAsync(&nj, njobs, 4, hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            const double w = (double)((nj + hj - 1) / hj);
            fprintf(stderr, "zstd huf kernel: %u sections, %.0f symbols a stream; per wave: intervals %.0f; clocks per "
                            "interval: uniform point %.0f (its wait %.0f), steps %.0f; inexact streams %llu (x1) %llu (x2), "
                            "far %llu\n",
                    nj, (double)h[4] / (nj ? 4.0 * nj : 1.0), h[2] / (w ? w : 1), (double)h[0] / (h[2] ? h[2] : 1),
                    (double)h[3] / (h[2] ? h[2] : 1), (double)h[1] / (h[2] ? h[2] : 1), h[5], h[6], h[7]);
        }
#endif
        unsigned long long* sstats = nullptr;
#if LZH_ZSTD_STATS
        static unsigned long long* d_sst = nullptr;
        if (!d_sst) (void)hipMalloc(&d_sst, 16 * sizeof(unsigned long long));
        (void)hipMemsetAsync(d_sst, 0, 16 * sizeof(unsigned long long), s);
        sstats = d_sst;
#endif
        if (!side)
            hipLaunchKernelGGL(lzh_zstd_seq_kernel, dim3(sgrid), dim3(64), 0, s, packed, packed_readable, offsets,
                               chunk_size, nchunks, status, zt, zst, zfr, sstats, (const uint32_t*)nullptr,
                               (const uint32_t*)nullptr, -1);
#if LZH_ZSTD_STATS
        {
            unsigned long long h[16];
            (void)hipMemcpyAsync(h, d_sst, sizeof(h), hipMemcpyDeviceToHost, s);
            (void)hipStreamSynchronize(s);
            const double w = (double)((nchunks + zsplit::kFPW - 1) / zsplit::kFPW);
            fprintf(stderr, "zstd seq kernel per wave: intervals %.0f (with block starts %.0f), steps %.0f; clocks per "
                            "interval: uniform point %.0f (its wait %.0f), steps %.0f; frames to the one-wave decoder %llu; clock %.0f MHz\n",
                    h[2] / w, h[3] / w, h[4] / w, (double)h[0] / h[2], (double)h[5] / h[2], (double)h[1] / h[2], h[6],
                    100.0 * (double)h[8] / (double)(h[9] ? h[9] : 1));
        }
#endif
        if (plan) {
            for (int k = 1; k >= 0; k--) {   // the short list once its sequences are done, then the long one
                (void)hipStreamWaitEvent(s, join[k], 0);
                hipLaunchKernelGGL(lzh_zstd_exec_kernel, dim3(nchunks), dim3(64), 0, s, packed, packed_readable, offsets,
                                   csizes, n_total, chunk_size, out, status, zt, zst, zfr, (const uint32_t*)flist,
                                   (const uint32_t*)fcnt, 1 - k, nchunks);
            }
        } else {
            if (side) (void)hipStreamWaitEvent(s, join[0], 0);
            hipLaunchKernelGGL(lzh_zstd_exec_kernel, dim3(nchunks), dim3(64), 0, s, packed, packed_readable, offsets,
                               csizes, n_total, chunk_size, out, status, zt, zst, zfr, (const uint32_t*)nullptr,
                               (const uint32_t*)nullptr, -1, nchunks);
        }
        zsel = zst;
    }
    hipLaunchKernelGGL(lzh_zstd_decompress_kernel, dim3(nchunks), dim3(64), 0, s, packed, packed_readable, offsets,
                       csizes, n_total, chunk_size, out, status, 0u, stats, zsel);
#if LZH_ZSTD_STATS
    unsigned long long h[zstdd::kZClk];
    (void)hipMemcpyAsync(h, d_stats, sizeof(h), hipMemcpyDeviceToHost, s);
    (void)hipStreamSynchronize(s);
    unsigned long long tot = 0;
    for (int i = 0; i < zstdd::kZClk; i++) tot += h[i];
    static const char* names[zstdd::kZClk] = {"headers", "huf_table", "huf_streams", "seq_tables", "seq_decode",
                                              "emit_group", "long_seq", "tail"};
    fprintf(stderr, "zstd clocks per chunk %.0f:", (double)tot / nchunks);
    for (int i = 0; i < zstdd::kZClk; i++) fprintf(stderr, " %s %.1f%%", names[i], 100.0 * h[i] / (tot ? tot : 1));
    fprintf(stderr, "\n");
#endif
    return hipGetLastError();
}

// bytes of the split decoder's temp for n bytes in chunks of chunk_size (per frame: blocks, block
// positions, sequence tables, sequences; then the frame states and frame fields)
// (0 below lzh_zstd_split_min: the layout reserves two block slots (~17 KiB) and 2 x chunk of sequence
// records per frame, 20x the input at 1 KiB chunks; small frames decode in the one-wave kernel)
size_t lzh_zstd_decode_temp(uint64_t n, uint64_t chunk_size) {
    if (chunk_size < lzh_zstd_split_min) return 0;
    const uint64_t k = (n + chunk_size - 1) / chunk_size;
    const zsplit::ZLayout Z = zsplit::zlayout(chunk_size);
    return k * Z.stride + zsplit::zdummy_bytes(k) + ((k * 4 + 255) & ~255ull) + ((k * sizeof(zsplit::ZFrame) + 255) & ~255ull) + 256 +
           k * Z.bmax * sizeof(zsplit::ZHuf) + 256 + ((k * 4 + 8 + 255) & ~255ull);   // (+ the plan's frame list, counts)
}
