// lzbench_amd/csrc/snappy_hip.hip -- snappy raw format for gfx950, bit-exact with snappy 1.1.8.
//
// One 64-lane wavefront per lzbench chunk.  The chunk is a varint32 length followed by the
// concatenation of independently compressed 64 KiB fragments (reference
// snappy/snappy.cc:1043-1111); each fragment gets a freshly zeroed LDS hash table of
// CalculateTableSize(fragment) u16 entries (<= 16384 = 32 KiB, snappy.cc:457-495).
// CompressFragment (snappy.cc:510-681) is parallelised like the LZ4 kernel: 64 probe
// positions of the search schedule per batch (16 unrolled probes, then the skip>>5
// heuristic, whose position sequence is data independent: skip grows by exactly the step,
// so skip - position is constant along a search), exact in-batch slot-collision
// resolution, and the post-copy re-test at ip (after inserting ip-1) as lane 0 of the next
// batch.
#include "common.h"

namespace {

struct SnTable {
    LDSA uint16_t* t;
    __device__ __forceinline__ uint32_t get(uint32_t h) const { return ((volatile const LDSA uint16_t*)t)[h]; }
    __device__ __forceinline__ void put(uint32_t h, uint32_t v) const { ((volatile LDSA uint16_t*)t)[h] = (uint16_t)v; }
};

__device__ __forceinline__ int log2floor_u(uint32_t v) { return 31 - __builtin_clz(v); }

__device__ __forceinline__ uint32_t sn_table_size(uint32_t n) {
    if (n > (1u << 14)) return 1u << 14;
    if (n < (1u << 8)) return 1u << 8;
    return 2u << log2floor_u(n - 1);
}

// u after i steps of u -> u + (u >> 5), walked one constant-step segment at a time
__device__ __forceinline__ uint32_t skip_walk(uint32_t u, int i) {
    for (int it = 0; it < 64 && i > 0; it++) {
        const uint32_t m = u >> 5;
        uint32_t t = (32u * (m + 1) - u + m - 1) / m;   // steps left with this step size
        if (t > (uint32_t)i) t = (uint32_t)i;
        u += t * m;
        i -= (int)t;
    }
    return u;
}

__device__ __forceinline__ void copy_bytes(const Bytes& in, int src, const Bytes& out, int dst, int len, int lane) {
    copy_span(in, src, out, dst, len, lane, LZH_WAVE);
}

// EmitLiteral (snappy.cc:342-383): tag (+1..4 length bytes), then the bytes. Returns new op.
__device__ __forceinline__ int emit_literal(const Bytes& in, int src, const Bytes& out, int op, int len, int lane) {
    const int nm1 = len - 1;
    if (nm1 < 60) {
        if (lane == 0) out.st8(op, (uint32_t)nm1 << 2);
        op += 1;
    } else {
        const int count = (log2floor_u((uint32_t)nm1) >> 3) + 1;
        if (lane == 0) out.st8(op, (uint32_t)(59 + count) << 2);
        if (lane >= 1 && lane <= count) out.st8(op + lane, ((uint32_t)nm1 >> (8 * (lane - 1))) & 0xffu);
        op += 1 + count;
    }
    copy_bytes(in, src, out, op, len, lane);
    return op + len;
}

// EmitCopy (snappy.cc:385-443): 64-byte COPY_2 pieces while len >= 68, one 60 if len > 64,
// then COPY_1 (len < 12 && offset < 2048) or COPY_2.  Returns new op.
__device__ __forceinline__ int emit_copy(const Bytes& out, int op, uint32_t off, int len, int lane) {
    int k = 0, has60 = 0, rem = len;
    if (len >= 12) {
        k = len >= 68 ? (len - 68) / 64 + 1 : 0;
        rem = len - 64 * k;
        if (rem > 64) { has60 = 1; rem -= 60; }
    }
    const bool c1 = rem < 12 && off < 2048u;
    const int pre = 3 * (k + has60);
    const int total = pre + (c1 ? 2 : 3);
    const uint32_t lo = off & 0xffu, hi = (off >> 8) & 0xffu;
    for (int base = 0; base < total; base += LZH_WAVE) {
        const int t = base + lane;
        if (t < total) {
            uint32_t v;
            if (t < pre) {
                const int piece = t / 3, b = t - 3 * piece;
                const uint32_t tag = (piece < k) ? (2u | (63u << 2)) : (2u | (59u << 2));
                v = b == 0 ? tag : (b == 1 ? lo : hi);
            } else {
                const int b = t - pre;
                if (c1) v = b == 0 ? (1u | ((uint32_t)(rem - 4) << 2) | ((off >> 8) << 5)) : lo;
                else v = b == 0 ? (2u | ((uint32_t)(rem - 1) << 2)) : (b == 1 ? lo : hi);
            }
            out.st8(op + t, v);
        }
    }
    return op + total;
}

// CompressFragment over in[0..fn) (in is the fragment's own descriptor); writes at op.
__device__ int sn_compress_fragment(const Bytes& in, int fn, const Bytes& out, int op, LDSA uint16_t* lds) {
    const int lane = threadIdx.x;
    SnTable T{lds};
    const uint32_t tsize = sn_table_size((uint32_t)fn);
    const int shift = 32 - log2floor_u(tsize);
    {
        LDSA uint32_t* t4 = (LDSA uint32_t*)lds;
        const int nvec = (int)(tsize * 2 / 16);
        for (int i = lane; i < nvec; i += LZH_WAVE) lds_zero16(t4 + 4 * i);
        wave_lds_fence();
    }
    int next_emit = 0;
    if (fn >= 15) {
        const int ip_limit = fn - 15;
        // search state: probes from q0 (after next_emit); unrolled block if ip_limit-q0 >= 16
        bool retest = false;
        int rt = 0;          // retest position (== next_emit) when retest
        int q0 = 1;          // first search position
        int t0 = 0;          // index of this batch's first search probe within the search
        // checked-probe reference state: probe index ci0 sits at position cq0 with skip cu0
        int ci0 = 0, cq0 = 0;
        uint32_t cu0 = 32;
        bool unrolled = ip_limit - q0 >= 16;
        if (unrolled) { cq0 = q0 + 16; cu0 = 48; } else { cq0 = q0; cu0 = 32; }
        next_emit = 0;
        for (int guard = 0; guard < 4 * fn + 64; guard++) {
            int64_t p;
            bool valid;
            uint32_t u = 0;
            int i = -1;
            if (retest && lane == 0) {
                p = rt;
                valid = true;
            } else {
                const int t = retest ? lane - 1 : t0 + lane;
                if (unrolled && t < 16) {
                    p = q0 + t;
                    valid = true;
                } else {
                    i = unrolled ? t - 16 : t;
                    u = skip_walk(cu0, i - ci0);          // 0 <= i - ci0 <= 63
                    p = (int64_t)cq0 + (int64_t)(u - cu0);
                    valid = p + (int64_t)(u >> 5) <= ip_limit;
                }
            }
            const int pos = valid ? (int)p : 0;
            const uint32_t pw = in.w32(pos);
            const uint32_t h = (pw * 0x1e35a7bdu) >> shift;
            const uint32_t old = T.get(h);
            if (valid) T.put(h, (uint32_t)pos);
            wave_lds_fence();
            const uint32_t back = T.get(h);
            const uint64_t dup = ballot(valid && back != (uint32_t)pos);
            uint32_t cand = old;
            uint64_t grp = 1ull << lane;
            if (dup) {
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
            const uint32_t cw = in.w32(valid ? (int)cand : 0);
            const bool ok = valid && cw == pw;
            const uint64_t hits = ballot(ok);
            const uint64_t inval = ballot(!valid);
            const int fh = ffs64(hits), fi = ffs64(inval);
            const bool found = hits != 0;
            const int L = found ? fh : fi - 1;
            if (!dup) {
                if (valid && lane > L) T.put(h, old);
            } else if (valid && lane <= L) {
                const uint64_t upto = (L >= 63) ? ~0ull : ((2ull << L) - 1ull);
                const uint64_t later = grp & ~((2ull << lane) - 1ull) & upto;
                if (!later) T.put(h, (uint32_t)pos);
            }
            wave_lds_fence();

            if (!found) {
                if (inval) break;          // search exhausted: remainder from next_emit
                {   // lane 63 is always a checked probe: next batch starts one step after it
                    const uint32_t u63 = rdlane(u, 63);
                    const int q63 = rdlanei(pos, 63);
                    ci0 = rdlanei(i, 63) + 1;
                    cq0 = q63 + (int)(u63 >> 5);
                    cu0 = u63 + (u63 >> 5);
                }
                if (retest) { retest = false; t0 = LZH_WAVE - 1; }
                else t0 += LZH_WAVE;
                continue;
            }
            int ip = rdlanei(pos, fh);
            int cpos = rdlanei((int)cand, fh);
            if (ip > next_emit) op = emit_literal(in, next_emit, out, op, ip - next_emit, lane);

            // copy: FindMatchLength(candidate + 4, ip + 4, ip_end)
            const int a = ip + 4, b = cpos + 4;
            int len = 0;
            for (int it = 0; it < (1 << 11) && a + len < fn; it++) {
                const int o = len + 4 * lane;
                const uint32_t x = in.w32(a + o) ^ in.w32(b + o);
                const uint64_t ne = ballot(x != 0);
                if (ne) {
                    const int l = ffs64(ne);
                    len += 4 * l + (__builtin_ctz(rdlane(x, l)) >> 3);
                    break;
                }
                len += 4 * LZH_WAVE;
            }
            len = min(len, fn - a);
            const int matched = 4 + len;
            op = emit_copy(out, op, (uint32_t)(ip - cpos), matched, lane);
            ip += matched;
            next_emit = ip;
            if (ip >= ip_limit) break;
            {   // insert ip-1, then re-test ip as lane 0 of the next batch
                const uint32_t w = in.w32(ip - 1);
                const uint32_t hm1 = (w * 0x1e35a7bdu) >> shift;
                if (lane == 0) T.put(hm1, (uint32_t)(ip - 1));
                wave_lds_fence();
            }
            retest = true;
            rt = ip;
            q0 = ip + 1;
            t0 = 0;
            unrolled = ip_limit - q0 >= 16;
            ci0 = 0;
            if (unrolled) { cq0 = q0 + 16; cu0 = 48; } else { cq0 = q0; cu0 = 32; }
        }
    }
    if (next_emit < fn) op = emit_literal(in, next_emit, out, op, fn - next_emit, lane);
    return op;
}

}  // namespace

extern "C" __global__ void __launch_bounds__(64)
lzh_snappy_compress_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                           uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t chunk0) {
    __shared__ __attribute__((aligned(16))) uint16_t lds[1 << 14];
    const int lane = threadIdx.x;
    const uint64_t chunk = (uint64_t)blockIdx.x + chunk0;
    const uint64_t off = chunk * chunk_size;
    if (off >= n_total && !(n_total == 0 && chunk == 0)) return;
    const uint32_t n = (uint32_t)min(chunk_size, n_total - off);
    Bytes rout;
    rout.init(stage + chunk * stride, stride);
    // varint32 uncompressed length
    int op = 0;
    {
        uint32_t v = n;
        int nb = 1;
        while (v >= 128) { v >>= 7; nb++; }
        if (lane < nb) {
            const uint32_t byte = (n >> (7 * lane)) & 0x7fu;
            rout.st8(lane, byte | (lane + 1 < nb ? 0x80u : 0u));
        }
        op = nb;
    }
    for (uint32_t fpos = 0; fpos < n; fpos += 65536u) {
        const int fn = (int)min(65536u, n - fpos);
        const uint64_t readable = min<uint64_t>(in_readable - off - fpos, (uint64_t)fn + 64);
        Bytes rin;
        rin.init(in + off + fpos, readable);
        op = sn_compress_fragment(rin, fn, rout, op, (LDSA uint16_t*)lds);
    }
    if (lane == 0) csizes[chunk] = (uint32_t)op;
}

#include "launch.h"
hipError_t lzh_launch_snappy_compress(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                      uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks,
                                      hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(lzh_snappy_compress_kernel, dim3(nchunks), dim3(64), 0, s, in, n_total, in_readable,
                       chunk_size, stage, stride, csizes, 0u);
    return hipGetLastError();
}
