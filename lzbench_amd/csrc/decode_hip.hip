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

namespace {


struct Win {
    rsrc_t r;
    int sh;       // descriptor offset of stream byte 0
    int wb;       // descriptor offset (4-aligned) of the window start
    uint32_t w0, w1;
    __device__ __forceinline__ void bind(const Bytes& b) { r = b.r; sh = b.sh; }
    __device__ __forceinline__ void load(int pos, int lane) {
        wb = (pos + sh) & ~3;
        w0 = ld_b32(r, wb + 4 * lane);
        w1 = ld_b32(r, wb + 256 + 4 * lane);
    }
    // make stream bytes [pos, pos+16) addressable
    __device__ __forceinline__ void ensure(int pos, int lane) {
        const int x = pos + sh;
        if (x >= wb && x + 16 <= wb + 512) return;
        if (x >= wb + 256 && x + 16 <= wb + 768) {
            w0 = w1;
            wb += 256;
            w1 = ld_b32(r, wb + 256 + 4 * lane);
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
        const int d = (x - wb) >> 2;
        const uint32_t a0 = lane_gather(w0, d & 63), a1 = lane_gather(w1, d & 63);
        const uint32_t b0 = lane_gather(w0, (d + 1) & 63), b1 = lane_gather(w1, (d + 1) & 63);
        const uint32_t lo = d < 64 ? a0 : a1, hi = d + 1 < 64 ? b0 : b1;
        return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)x & 3u);
    }
    // per-lane byte at stream position pos (inside the window) via cross-lane permute
    __device__ __forceinline__ uint32_t lane_byte(int pos) const {
        const int x = pos + sh;
        const int d = (x - wb) >> 2;
        const uint32_t a = lane_gather(w0, d & 63), b = lane_gather(w1, d & 63);
        return ((d < 64 ? a : b) >> (8 * (x & 3))) & 0xffu;
    }
};

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
constexpr int kW = LZH_DEC_KW;   // LDS output window bytes (power of two)

struct Sink {
    LDSA uint8_t* b;
    Bytes out;
    int flushed;      // output bytes [0, flushed) are in global memory
    int ringlo;       // output bytes [ringlo, op) are in the window (bulk literal runs bypass it)
    __device__ __forceinline__ void put(int pos, uint32_t v) const {
        ((volatile LDSA uint8_t*)b)[(pos + out.sh) & (kW - 1)] = (uint8_t)v;
    }
    __device__ __forceinline__ uint32_t get(int pos) const {
        return ((volatile const LDSA uint8_t*)b)[(pos + out.sh) & (kW - 1)];
    }
    __device__ __forceinline__ uint32_t dword(int X) const {
        return ((volatile const LDSA uint32_t*)b)[(X & (kW - 1)) >> 2];
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
    __device__ __forceinline__ void literals(const Win& w, const Bytes& in, int src, int op, int len, int lane) {
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
        if (src0 >= ringlo && off <= kW - LZH_WAVE) {
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

}  // namespace owin

// ---------------------------------------------------------------------------------------
// One LZ4 sequence at a time with every acceptance rule of LZ4_decompress_safe (lz4.c:1707-1729,
// :1929-2151): the path for what a group does not take (255-run lengths, the last-literals
// sequence, malformed input).  Returns 0 = continue, 1 = done (last literals), < 0 = error.
namespace checked {

using owin::kW;

__device__ __forceinline__ int lz4_one(const Bytes& in, int cs, owin::Sink& O, Win& w, int cap, int& ip, int& op,
                                       int lane) {
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
    if (off > op) return -ip - 1;
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

// Assemble a group's output [op, op + total): sequence k (member lane k, output start excl) is
// litk literal bytes from stream position ip + lrel, then mlk match bytes copied from offset offk
// (byte-by-byte semantics); a literal-only member has mlk = 0, a copy-only member litk = 0.
// One output byte per lane per pass; the owner is the last start mark at or before the byte.
__device__ __forceinline__ void emit_group(const Win& w, owin::Sink& O, LDSA uint8_t* mark, int ip, int op,
                                           int total, uint64_t keep, int excl, uint32_t pA, uint32_t lrel,
                                           int off, int lane) {
    const bool kmem = (keep >> lane) & 1ull;
    int carry = 63 - __builtin_clzll(keep);                      // (pass 0 always has a start at 0)
    // Branch-free pass body: lanes that have nothing to store write to harmless places (the mark
    // scratch's second half, or output bytes past `total` / of this pass that a later round or
    // group overwrites before any flush), so no exec-mask juggling per conditional access.
    for (int pass = 0; pass * LZH_WAVE < total; pass++) {
        const int pb = pass * LZH_WAVE;
        mark[lane] = 0xff;
        wave_lds_fence();
        const bool mine = kmem && excl >= pb && excl < pb + LZH_WAVE;
        mark[mine ? excl - pb : LZH_WAVE + lane] = (uint8_t)lane;
        wave_lds_fence();
        const int mv = (int)mark[lane];
        const uint64_t S = ballot(mv != 0xff);
        const uint64_t le = S & ((2ull << lane) - 1ull);
        const int js = le ? 63 - __builtin_clzll(le) : lane;
        const int own_here = (int)lane_gather((uint32_t)mv, js);
        const int k = le ? own_here : carry;
        carry = rdlanei(k, 63);
        const uint32_t a = lane_gather(pA, k), b = lane_gather(lrel, k);
        const int ek = (int)lane_gather((uint32_t)excl, k);
        const int offk = (int)lane_gather((uint32_t)off, k);
        const int litk = (int)(a & 0xffffu);
        const int ob = pb + lane;
        const bool act = ob < total;
        const int u = ob - ek;
        const bool is_lit = u < litk;
        const uint32_t lb = w.lane_byte(ip + (int)b + (is_lit ? u : 0));
        const int mu = u - litk;
        const int mstart = op + ek + litk;
        int src = mstart - offk + mu;
        if (ballot(act && !is_lit && mu >= offk)) {                // overlapping copy: period offk
            const int md = (int)((uint32_t)mu % (uint32_t)max(offk, 1));
            src = (!is_lit && mu >= offk) ? mstart - offk + md : src;
        }
        const int pbase = op + pb;
        const bool near = !is_lit && src >= O.ringlo && src >= pbase + LZH_WAVE - kW;
        const bool inpass = !is_lit && src >= pbase;
        const uint32_t g = O.get(src);
        uint32_t v = is_lit ? lb : g;
        bool done = is_lit || (near && !inpass);
        const bool far = act && !is_lit && !near;
        if (ballot(far)) {   // far sources were flushed long ago: their stores must be done
            wait_vm();
            const uint32_t gv = O.out.b_sc1(far ? src : 0);
            v = far ? gv : v;
            done = done || far;
        }
        O.put(op + ob, v);
        uint64_t dm = ballot(act && done) | ~ballot(act);
        for (int r = 0; r < LZH_WAVE && ~dm; r++) {
            const int sl = src - pbase;
            const bool ready = !((dm >> lane) & 1ull) && ((dm >> (sl & 63)) & 1ull);
            const uint32_t vv = O.get(src);
            v = ready ? vv : v;
            O.put(op + ob, v);
            dm |= ballot(ready);
        }
        O.maybe_flush(min(pbase + LZH_WAVE, op + total), lane);
    }
}

// Lanes on the chain that starts at lane 0 and follows `link` (next lane, strictly increasing;
// >= 64 = leaves the group, 255 = the lane itself is not taken), by binary lifting: jump tables
// J_k = link^(2^k) through ds_bpermute, then every lane lifts from lane 0 to the furthest chain
// lane <= itself.  No scalar walk (the decoder is scalar-issue bound).
__device__ __forceinline__ uint64_t chain_members(int link, int lane) {
    const int J0 = min(link, LZH_WAVE);
    const int J1 = J0 < LZH_WAVE ? (int)lane_gather((uint32_t)J0, J0) : LZH_WAVE;
    const int J2 = J1 < LZH_WAVE ? (int)lane_gather((uint32_t)J1, J1) : LZH_WAVE;
    const int J3 = J2 < LZH_WAVE ? (int)lane_gather((uint32_t)J2, J2) : LZH_WAVE;
    const int J4 = J3 < LZH_WAVE ? (int)lane_gather((uint32_t)J3, J3) : LZH_WAVE;
    const int J5 = J4 < LZH_WAVE ? (int)lane_gather((uint32_t)J4, J4) : LZH_WAVE;
    int x = 0, y;
    y = (int)lane_gather((uint32_t)J5, x); x = y <= lane ? y : x;
    y = (int)lane_gather((uint32_t)J4, x); x = y <= lane ? y : x;
    y = (int)lane_gather((uint32_t)J3, x); x = y <= lane ? y : x;
    y = (int)lane_gather((uint32_t)J2, x); x = y <= lane ? y : x;
    y = (int)lane_gather((uint32_t)J1, x); x = y <= lane ? y : x;
    y = (int)lane_gather((uint32_t)J0, x); x = y <= lane ? y : x;
    return ballot(x == lane && link != 255);
}

__device__ int lz4_decode(const Bytes& in, int cs, owin::Sink& O, LDSA uint8_t* mark, int cap, int lane) {
    if (cap == 0) return (cs == 1 && in.b(0) == 0) ? 0 : -1;
    if (cs <= 0) return -1;
    Win w;
    w.bind(in);
    w.load(0, lane);
    int ip = 0, op = 0;
    for (int guard = 0; guard <= cs; guard++) {
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
        const uint64_t M = chain_members(link, lane);
        // ---- acceptance rules per member (as lz4_one); the chain ends before the first failure
        const bool mem = (M >> lane) & 1ull;
        const int L = mem ? lit + ml : 0;
        const int incl = wave_incl_scan(L);
        const int excl = incl - L;
        const int opm = op + excl + lit;
        const bool bad = mem && (x >= cs || (ln == 15 && x + 1 >= cs - 15) || opm > cap - 12 || p1 + lit > cs - 8 ||
                                 (mc == 15 && po + 3 >= cs - 4) || off == 0 || off > opm || opm + ml > cap - 5);
        const uint64_t badm = ballot(bad);
        const uint64_t keep = badm ? (M & ((1ull << __builtin_ctzll(badm)) - 1ull)) : M;
        if (!keep) {
            const int r = checked::lz4_one(in, cs, O, w, cap, ip, op, lane);
            if (r < 0) return r;
            if (r == 1) break;
            continue;
        }
        const int lastk = 63 - __builtin_clzll(keep);
        const int total = rdlanei(incl, lastk);
        const int ip_next = ip + rdlanei(pe - ip, lastk);
        emit_group(w, O, mark, ip, op, total, keep, excl, (uint32_t)lit | ((uint32_t)ml << 16), (uint32_t)(p1 - ip),
                   off, lane);
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
__device__ int snappy_decode(const Bytes& in, int cs, owin::Sink& O, LDSA uint8_t* mark, int cap, int lane) {
    Win w;
    w.bind(in);
    w.load(0, lane);
    int ip = 0;
    uint32_t ulen = 0;
    for (int shift = 0;; shift += 7) {
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
        const bool mem = (M >> lane) & 1ull;
        const int L = mem ? len : 0;
        const int incl = wave_incl_scan(L);
        const int excl = incl - L;
        const int opm = op + excl;
        const bool bad = mem && (x >= cs || !okr || opm + len > ul || (kind != 0 && off > opm));
        const uint64_t badm = ballot(bad);
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

extern "C" __global__ void __launch_bounds__(64)
lzh_decompress_v2_kernel(int codec, const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                         const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint8_t* out,
                         int32_t* status, uint32_t chunk0) {
    __shared__ __attribute__((aligned(16))) uint8_t win[owin::kW + 2 * LZH_WAVE];   // output window | start marks
    const int lane = threadIdx.x;
    const uint64_t chunk = (uint64_t)blockIdx.x + chunk0;
    const uint64_t ooff = chunk * chunk_size;
    if (ooff >= n_total) return;
    const int part = (int)min(chunk_size, n_total - ooff);
    const uint64_t ioff = offsets[chunk];
    const int cs = (int)csizes[chunk];
    const uint64_t readable = ioff < packed_readable ? min<uint64_t>(packed_readable - ioff, (uint64_t)cs + 16) : 0;
    Bytes rin, rout;
    rin.init(packed + ioff, readable);
    rout.init(out + ooff, (uint64_t)part);
    int r;
    if (cs == part || codec == 2) {
        copy_raw(rin, rout, part, lane);
        r = part;
    } else {
        owin::Sink O{(LDSA uint8_t*)win, rout, 0, 0};
        r = codec == 0 ? groups::lz4_decode(rin, cs, O, (LDSA uint8_t*)win + owin::kW, part, lane)
                       : groups::snappy_decode(rin, cs, O, (LDSA uint8_t*)win + owin::kW, part, lane);
        if (r > 0) O.flush(r, lane);
    }
    if (lane == 0) status[chunk] = r;
}

#include "launch.h"
hipError_t lzh_launch_decompress(int codec, const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                                 const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint8_t* out,
                                 int32_t* status, uint32_t nchunks, hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(lzh_decompress_v2_kernel, dim3(nchunks), dim3(64), 0, s, codec, packed, packed_readable,
                       offsets, csizes, n_total, chunk_size, out, status, 0u);
    return hipGetLastError();
}
