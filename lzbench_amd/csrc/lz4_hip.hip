// lzbench_amd/csrc/lz4_hip.hip -- LZ4 block codec for gfx950, bit-exact with lz4 1.9.3.
//
// One 64-lane wavefront (one workgroup) per lzbench chunk; the chunk's hash table lives in
// LDS (16 KiB: 8192 x u16 for chunks < 65547 B "byU16", 4096 x u32 "byU32" otherwise,
// reference lz4/lz4.c:633, :1284-1305).  The greedy parse of LZ4_compress_generic
// (lz4.c:851-1240) is inherently sequential; the wave parallelises *within* each step:
//
//   * probe batch: the 64 lanes take the next 64 probe positions of the search schedule
//     (step = searchMatchNb++ >> 6, lz4.c:954-1014; positions are data independent), hash
//     them, read the table, and resolve "an earlier lane of this batch wrote the same
//     slot" exactly (write / read-back detection, exact group resolution on collision).
//     The first lane whose candidate matches ends the batch; only the table writes of the
//     lanes up to it are kept.  The immediate re-test at a match end (lz4.c:1145-1197) is
//     lane 0 of the following batch, lanes 1..63 continue with the search from ip+1.
//   * catch-up (lz4.c:1019), match length (LZ4_count, lz4.c:603-626) and literal copies
//     run 64 bytes per step with ballots.
//
// Output goes to a fixed-stride staging slot per chunk; packing is done by lzh_pack.
#include "common.h"

namespace {

constexpr int kMinMatch = 4;
constexpr int kMfLimit = 12;
constexpr int kLastLiterals = 5;
constexpr int kMinLength = 13;

// sum_{m < M} (m >> 6)
__device__ __forceinline__ int64_t step_prefix(int64_t M) {
    int64_t q = M >> 6, r = M & 63;
    return 32 * q * (q - 1) + r * q;
}

// probe k (0-based) of a search: offset from the search start and the step taken after it
__device__ __forceinline__ void probe_sched(int k, int64_t a64, int64_t& off, int64_t& step) {
    if (k == 0) { off = 0; step = 1; return; }
    off = 1 + step_prefix(a64 + k - 1) - step_prefix(a64);
    step = (a64 + k - 1) >> 6;
}

// table accesses are volatile: other lanes of the wave write the same slots, so the
// compiler must neither forward a lane's own store nor cache a slot in a register
template <bool kSmall>
struct Lz4Table {
    LDSA uint32_t* raw;   // 16 KiB of LDS
    __device__ __forceinline__ uint32_t get(uint32_t h) const {
        if (kSmall) return ((volatile const LDSA uint16_t*)raw)[h];
        return ((volatile const LDSA uint32_t*)raw)[h];
    }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const {
        if (kSmall) ((volatile LDSA uint16_t*)raw)[h] = (uint16_t)v; else ((volatile LDSA uint32_t*)raw)[h] = v;
    }
};

template <bool kSmall>
__device__ __forceinline__ uint32_t lz4_hash_at(const Bytes& in, int pos, uint32_t& w32) {
    if (kSmall) {
        w32 = in.w32(pos);
        return (w32 * 2654435761u) >> 19;
    }
    uint64_t v = in.w40(pos);
    w32 = (uint32_t)v;
    return (uint32_t)(((v << 24) * 889523592379ull) >> 52);
}

// copy len bytes in -> out (byte granular, 4 bytes per lane per round, loads before stores)
__device__ __forceinline__ void copy_bytes(const Bytes& in, int src, const Bytes& out, int dst, int len, int lane) {
    copy_span(in, src, out, dst, len, lane, LZH_WAVE);
}

// write a length header: byte0 (token or 0), then the 255-run continuation of `ext` (if has_ext)
__device__ __forceinline__ int ext_len_bytes(int v) { return v >= 15 ? (v - 15) / 255 + 1 : 0; }

__device__ __forceinline__ void write_run(const Bytes& out, int dst, int count, int rem, int lane) {
    // count bytes: count-1 x 255 then rem
    for (int base = 0; base < count; base += LZH_WAVE) {
        int t = base + lane;
        if (t < count) out.st8(dst + t, t == count - 1 ? (uint32_t)rem : 255u);
    }
}

template <bool kSmall>
__device__ void lz4_compress_chunk(const Bytes& in, int n, const Bytes& out, int acc, LDSA uint32_t* lds,
                                   uint32_t* out_size) {
    const int lane = threadIdx.x;
    Lz4Table<kSmall> T{lds};
    int op = 0, anchor = 0;

    if (n <= 0) {
        if (lane == 0) out.st8(0, 0);
        if (lane == 0) *out_size = 1;
        return;
    }
    // zero the table: 16 KiB = 64 lanes x 16 x 16 B
    {
        LDSA uint32_t* t4 = (LDSA uint32_t*)lds;
#pragma unroll
        for (int i = 0; i < 16; i++) lds_zero16(t4 + 4 * (i * LZH_WAVE + lane));
        wave_lds_fence();
    }
    if (n >= kMinLength) {
        const int mfl1 = n - kMfLimit + 1;    // mflimitPlusOne
        const int mlimit = n - kLastLiterals;  // matchlimit
        const int64_t a64 = (int64_t)acc << 6;

        {   // first byte
            uint32_t w;
            uint32_t h0 = lz4_hash_at<kSmall>(in, 0, w);
            if (lane == 0) T.put(h0, 0);
            wave_lds_fence();
        }
        int ip = 1;          // retest: position under re-test; search: unused
        int s = 1, k0 = 0;   // search start and first probe index of this batch
        bool retest = false;

        // every iteration of this loop consumes at least one probe position, bound it
        for (int guard = 0; guard < 4 * n + 64; guard++) {
            // ---- probe plan for this batch
            int64_t p, nxt;
            if (retest && lane == 0) {
                p = ip;
                nxt = (int64_t)ip + 1;
            } else {
                int k = retest ? lane - 1 : k0 + lane;
                int64_t o, st;
                probe_sched(k, a64, o, st);
                p = (int64_t)s + o;
                nxt = p + st;
            }
            const bool valid = nxt <= mfl1;
            const int pos = valid ? (int)p : 0;
            uint32_t pw;
            const uint32_t h = lz4_hash_at<kSmall>(in, pos, pw);
            const uint32_t old = T.get(h);
            if (valid) T.put(h, (uint32_t)pos);
            wave_lds_fence();
            const uint32_t back = T.get(h);
            const uint64_t dup = ballot(valid && back != (uint32_t)pos);
            uint32_t cand = old;
            uint64_t grp = 1ull << lane;
            if (dup) {
                // exact resolution: candidate = position of the latest earlier lane with
                // the same hash, else the pre-batch table value
                wave_lds_fence();
                if (valid) T.put(h, old);
                wave_lds_fence();
                uint64_t pending = dup;
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
                const uint32_t ppos = lane_gather((uint32_t)pos, prev < 0 ? lane : prev);
                if (prev >= 0) cand = ppos;
            }
            bool ok = valid;
            if (!kSmall) ok = ok && (cand + 65535u >= (uint32_t)pos);
            const uint32_t cw = in.w32(ok ? (int)cand : 0);
            ok = ok && cw == pw;
            const uint64_t hits = ballot(ok);
            const uint64_t inval = ballot(!valid);
            const int fh = ffs64(hits), fi = ffs64(inval);
            const bool found = hits != 0;
            const int L = found ? fh : fi - 1;          // last lane whose table write stands
            if (!dup) {
                if (valid && lane > L) T.put(h, old);
            } else if (valid && lane <= L) {
                const uint64_t upto = (L >= 63) ? ~0ull : ((2ull << L) - 1ull);
                const uint64_t later = grp & ~((2ull << lane) - 1ull) & upto;
                if (lane == 63 || !later) T.put(h, (uint32_t)pos);
            }
            wave_lds_fence();

            if (!found) {
                if (inval) break;                        // ran past mflimit: last literals
                if (retest) { retest = false; s = ip + 1; k0 = LZH_WAVE - 1; }
                else k0 += LZH_WAVE;
                continue;
            }

            // ---- a match: catch up backwards (no-op for a lane-0 re-test hit: ip == anchor)
            int mpos = rdlanei((int)cand, fh);
            ip = rdlanei(pos, fh);
            for (int it = 0; it < (1 << 12); it++) {
                const int maxb = min(ip - anchor, mpos);
                if (maxb <= 0) break;
                const bool eq = lane < maxb && in.b(ip - 1 - lane) == in.b(mpos - 1 - lane);
                const uint64_t ne = ballot(!eq);
                const int b = ffs64(ne);
                ip -= b;
                mpos -= b;
                if (b < LZH_WAVE) break;
            }
            const int lit = ip - anchor;
            const int offset = ip - mpos;

            // ---- match length: LZ4_count(ip+4, match+4, matchlimit)
            const int a = ip + kMinMatch, bb = mpos + kMinMatch;
            int len = 0;
            for (int it = 0; it < (1 << 10) && a + len < mlimit; it++) {
                const int o = len + 4 * lane;
                const uint32_t x = in.w32(a + o) ^ in.w32(bb + o);
                const uint64_t ne = ballot(x != 0);
                if (ne) {
                    const int l = ffs64(ne);
                    const uint32_t xl = rdlane(x, l);
                    len += 4 * l + (__builtin_ctz(xl) >> 3);
                    break;
                }
                len += 4 * LZH_WAVE;
            }
            const int ml = min(len, mlimit - a);

            // ---- emit: token, literal length run, literals, offset, match length run
            const int lx = ext_len_bytes(lit), mx = ext_len_bytes(ml);
            const uint32_t token = ((uint32_t)min(lit, 15) << 4) | (uint32_t)min(ml, 15);
            if (lane == 0) out.st8(op, token);
            if (lx) write_run(out, op + 1, lx, (lit - 15) % 255, lane);
            copy_bytes(in, anchor, out, op + 1 + lx, lit, lane);
            const int tail = op + 1 + lx + lit;
            if (lane == 0) out.st8(tail, (uint32_t)offset & 0xffu);
            if (lane == 1) out.st8(tail + 1, (uint32_t)offset >> 8);
            if (mx) write_run(out, tail + 2, mx, (ml - 15) % 255, lane);
            op = tail + 2 + mx;

            ip = a + ml;
            anchor = ip;
            if (ip >= mfl1) break;
            {   // fill table at ip-2, then re-test ip as lane 0 of the next batch
                uint32_t w;
                const uint32_t hm2 = lz4_hash_at<kSmall>(in, ip - 2, w);
                if (lane == 0) T.put(hm2, (uint32_t)(ip - 2));
                wave_lds_fence();
            }
            retest = true;
            s = ip + 1;
            k0 = 0;
        }
    }
    // ---- last literals
    {
        const int run = n - anchor;
        const int rx = ext_len_bytes(run);
        if (lane == 0) out.st8(op, (uint32_t)min(run, 15) << 4);
        if (rx) write_run(out, op + 1, rx, (run - 15) % 255, lane);
        copy_bytes(in, anchor, out, op + 1 + rx, run, lane);
        op += 1 + rx + run;
    }
    if (lane == 0) *out_size = (uint32_t)op;
}

}  // namespace

// in: whole input (n_total bytes, readable up to in_readable); chunk i -> stage + i*stride
extern "C" __global__ void __launch_bounds__(64)
lzh_lz4_compress_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                        int acc, uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t chunk0) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[4096];
    const uint64_t chunk = (uint64_t)blockIdx.x + chunk0;
    const uint64_t off = chunk * chunk_size;
    if (off >= n_total && !(n_total == 0 && chunk == 0)) return;
    const int n = (int)min(chunk_size, n_total - off);
    const uint64_t readable = min<uint64_t>(in_readable - off, (uint64_t)n + 64);
    Bytes rin, rout;
    rin.init(in + off, readable);
    rout.init(stage + chunk * stride, stride);
    if (n < 65547) lz4_compress_chunk<true>(rin, n, rout, acc, (LDSA uint32_t*)lds, csizes + chunk);
    else lz4_compress_chunk<false>(rin, n, rout, acc, (LDSA uint32_t*)lds, csizes + chunk);
}

#include "launch.h"
hipError_t lzh_launch_lz4_compress(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                   int acc, uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks,
                                   hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(lzh_lz4_compress_kernel, dim3(nchunks), dim3(64), 0, s, in, n_total, in_readable,
                       chunk_size, acc, stage, stride, csizes, 0u);
    return hipGetLastError();
}
