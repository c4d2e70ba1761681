// lzbench_amd/csrc/frame_hip.hip -- framed LZ4 layouts on gfx950:
//
//   LZH_CODEC_LZ4F   one LZ4 frame per chunk, as LZ4F_compressFrame writes it with independent
//                    blocks (reference lz4/lz4frame.c:373-419 compressFrame, :598-700 header,
//                    :740-763 makeBlock, :825-927 / :986-1019 blocks, end mark, content checksum)
//   LZH_CODEC_NVLZ4  one nvcomp LZ4 container per chunk, the format of the reference's nvcomp_lz4
//                    row (nvcomp/LZ4Metadata.h:39-60: [4, metadata bytes, size, chunk size,
//                    offsets[0..k]] as 8-byte fields, LZ4CompressionKernels.cu:1038-1097: offsets
//                    are prefix sums from the metadata size, chunk streams back to back)
//
// Compression reuses the LZ4 block kernels (lz4c_hip.hip) over the frames' blocks -- a frame of
// F bytes is cut into ceil(F / B) blocks of B bytes (block_span) -- and then, per frame:
//   lzh_frame_size_kernel   one lane per frame: the frame's size from its blocks' sizes and the
//                           block offsets inside the frame; lzbench's raw-store rule on the frame
//   (lzh_scan_kernel)       frame offsets
//   lzh_frame_pack_kernel   one workgroup per block (header word, stored bytes, block checksum)
//                           and one per frame (frame header / end mark / content checksum, or the
//                           container header; a raw-stored frame is copied here)
// A block is stored raw exactly when its LZ4 block is not smaller than the block: LZ4F_makeBlock
// compresses with dstCapacity = size - 1 in limitedOutput mode (lz4.c:1316-1351), and since every
// sequence is followed by at least LASTLITERALS + 1 = 6 bytes (the match limit, lz4.c:883-884),
// the per-sequence checks (lz4.c:1097-1121) fail only when the last-literals check does
// (lz4.c:1207-1216), i.e. when the whole block does not fit: csize > size - 1.  (The CPU checker
// walks the checks themselves, and the tests compare against the reference's own LZ4F build.)
//
// Decompression: lzh_frame_parse_kernel (one wave per frame: header checks, block walk, block
// checksums) writes one 32-byte descriptor per block for the block decoder (decode_hip.hip,
// descriptor mode); lzh_frame_finish_kernel checks the blocks' results and the content checksum.
// XXH32 restates /root/reference/lz4/xxhash.c:269-389 as wave-uniform code.
#include "common.h"

namespace frm {

constexpr uint32_t P1 = 2654435761U, P2 = 2246822519U, P3 = 3266489917U, P4 = 668265263U, P5 = 374761393U;
__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// XXH32 (seed 0) of bytes [0, len) of b, computed by the whole wave: lane j loads 16-byte stripe j
// of each 1 KiB batch, the four accumulators then take the stripes in order (wave-uniform code)
__device__ uint32_t xxh32_wave(const Bytes& b, uint32_t len, int lane) {
    uint32_t h;
    uint32_t p = 0;
    if (len >= 16) {
        uint32_t v1 = P1 + P2, v2 = P2, v3 = 0, v4 = 0u - P1;
        const uint32_t ns = len / 16;   // stripes with p < len - 15, i.e. floor(len / 16)
        for (uint32_t s0 = 0; s0 < ns; s0 += 64) {
            const uint32_t q = (s0 + (uint32_t)lane) * 16;
            const bool in = s0 + (uint32_t)lane < ns;
            const uint32_t w0 = in ? b.w32(q) : 0, w1 = in ? b.w32(q + 4) : 0, w2 = in ? b.w32(q + 8) : 0,
                           w3 = in ? b.w32(q + 12) : 0;
            const uint32_t m = min(64u, ns - s0);
            for (uint32_t j = 0; j < m; j++) {
                v1 = rotl(v1 + rdlane(w0, (int)j) * P2, 13) * P1;
                v2 = rotl(v2 + rdlane(w1, (int)j) * P2, 13) * P1;
                v3 = rotl(v3 + rdlane(w2, (int)j) * P2, 13) * P1;
                v4 = rotl(v4 + rdlane(w3, (int)j) * P2, 13) * P1;
            }
        }
        p = ns * 16;
        h = rotl(v1, 1) + rotl(v2, 7) + rotl(v3, 12) + rotl(v4, 18);
    } else {
        h = P5;
    }
    h += len;
    const uint32_t t = b.w32((int)p), t2 = b.w32((int)p + 4), t3 = b.w32((int)p + 8), t4 = b.w32((int)p + 12);
    const uint32_t tw[4] = {uni(t), uni(t2), uni(t3), uni(t4)};
    int k = 0;
    for (; p + 4 <= len; p += 4, k++) h = rotl(h + tw[k] * P3, 17) * P4;
    for (; p < len; p++) h = rotl(h + uni(b.b((int)p)) * P5, 11) * P1;   // (bytewise: exact-size views)
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

__device__ __forceinline__ uint64_t bsize_of(int id) { return (uint64_t)1 << (8 + 2 * id); }

// LZ4F_optimalBSID (lz4frame.c:304-316); 0 = default = max64KB (lz4frame.c:640-641)
__device__ __forceinline__ int optimal_bsid(int req, uint64_t n) {
    int id = 4;
    uint64_t mb = 64u << 10;
    while (req > id) {
        if (n <= mb) return id;
        id++;
        mb <<= 2;
    }
    return req ? req : 4;
}

// little-endian byte stores of v at pos (a frame header field at an arbitrary byte offset)
__device__ __forceinline__ void put_le(const Bytes& o, int pos, uint64_t v, int nb) {
    for (int i = 0; i < nb; i++) o.st8(pos + i, (uint32_t)(v >> (8 * i)) & 0xffu);
}

}  // namespace frm

// LZ4F: frame header bytes for frame content size s
__device__ __forceinline__ int lz4f_header_len(int params, uint64_t s) { return 7 + (((params & 0x40) && s) ? 8 : 0); }

// one lane per frame: frame sizes (-> csizes[f], raw-store rule applied) and the offsets of the
// blocks inside their frame (rel[i]: LZ4F = the block's header word, NVLZ4 = its stream)
extern "C" __global__ void __launch_bounds__(256)
lzh_frame_size_kernel(int codec, int params, uint64_t n_total, uint64_t fs, uint64_t bs, uint32_t bpf,
                      const uint32_t* bcs, uint32_t* rel, uint32_t* csizes, uint32_t nframes) {
    const uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nframes) return;
    const uint64_t foff = f * fs;
    const uint64_t s = n_total > foff ? min(fs, n_total - foff) : 0;
    const uint32_t nb = (uint32_t)((s + bs - 1) / bs);
    uint64_t pos;
    if (codec == 4) {   // LZH_CODEC_LZ4F
        const int bcrc = (params >> 4) & 1, ccrc = (params >> 5) & 1;
        pos = (uint64_t)lz4f_header_len(params, s);
        for (uint32_t b = 0; b < nb; b++) {
            const uint64_t i = f * bpf + b;
            const uint32_t bsz = (uint32_t)min(bs, s - b * bs);
            const uint32_t c = bcs[i];
            rel[i] = (uint32_t)pos;
            pos += 4 + (c >= bsz ? bsz : c) + 4 * bcrc;
        }
        pos += 4 + 4 * ccrc;
    } else {            // LZH_CODEC_NVLZ4
        pos = 32 + 8 * ((uint64_t)nb + 1);
        for (uint32_t b = 0; b < nb; b++) {
            const uint64_t i = f * bpf + b;
            rel[i] = (uint32_t)pos;
            pos += bcs[i];
        }
    }
    csizes[f] = pos == s ? (uint32_t)s : (uint32_t)pos;   // lzbench.cpp:284-288: clen == part -> raw
}

// workgroups [0, nblocks): one block each; [nblocks, nblocks + nframes): one frame each
extern "C" __global__ void __launch_bounds__(256)
lzh_frame_pack_kernel(int codec, int params, const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t fs,
                      uint64_t bs, uint32_t bpf, const uint8_t* stage, uint64_t stride, const uint32_t* bcs,
                      const uint32_t* rel, const uint32_t* csizes, const uint64_t* offsets, uint8_t* packed,
                      uint32_t nblocks) {
    const int t = threadIdx.x;
    const uint64_t w = blockIdx.x;
    const bool lz4f = codec == 4;
    if (w < nblocks) {
        uint64_t boff;
        int bn;
        if (!block_span(w, n_total, bs, fs, bpf, boff, bn)) return;
        const uint64_t f = w / bpf, b = w - f * bpf;
        const uint64_t foff = f * fs, s = min(fs, n_total - foff);
        if (csizes[f] == s) return;   // frame stored raw
        const uint32_t c = bcs[w];
        const bool raw = lz4f && c >= (uint32_t)bn;
        const uint32_t st = raw ? (uint32_t)bn : c;
        const uint64_t dpos = offsets[f] + rel[w];
        Bytes src, dst;
        if (raw) src.init(in + boff, min<uint64_t>(in_readable - boff, (uint64_t)bn + 16));
        else src.init(stage + w * stride, stride);
        const int hb = lz4f ? 4 : 0, cb = lz4f && ((params >> 4) & 1) ? 4 : 0;
        dst.init(packed + dpos, (uint64_t)hb + st + cb);
        copy_span(src, 0, dst, hb, (int)st, t, blockDim.x);
        if (lz4f) {
            if (t == 0) frm::put_le(dst, 0, (uint64_t)(st | (raw ? 0x80000000u : 0u)), 4);
            if (cb && t < 64) {   // block checksum of the stored bytes (lz4frame.c:758-761)
                const uint32_t h = frm::xxh32_wave(src, st, t);
                if (t == 0) frm::put_le(dst, hb + (int)st, h, 4);
            }
        } else if (t == 0) {      // the container's offset entry of this chunk
            Bytes fr;
            fr.init(packed + offsets[f], 32 + 8 * (b + 1));
            frm::put_le(fr, 32 + 8 * (int)b, rel[w], 8);
        }
        return;
    }
    const uint64_t f = w - nblocks;
    const uint64_t foff = f * fs;
    if (foff >= n_total && !(n_total == 0 && f == 0)) return;
    const uint64_t s = n_total > foff ? min(fs, n_total - foff) : 0;
    const uint32_t fsz = csizes[f];
    Bytes dst;
    dst.init(packed + offsets[f], fsz);
    if (fsz == s) {   // raw-stored frame
        Bytes src;
        src.init(in + foff, min<uint64_t>(in_readable - foff, s + 16));
        copy_span(src, 0, dst, 0, (int)s, t, blockDim.x);
        return;
    }
    if (t >= 64) return;
    const uint32_t nb = (uint32_t)((s + bs - 1) / bs);
    if (lz4f) {
        const int bcrc = (params >> 4) & 1, ccrc = (params >> 5) & 1, csz = (params & 0x40) && s;
        const int bsid = frm::optimal_bsid(params & 7, s);
        // header (lz4frame.c:669-696): magic, FLG (version 01, independent blocks, flags), BD, content
        // size, HC = second byte of XXH32 of FLG..content size
        const uint32_t indep = (params & 0x80) && s > bs ? 0u : 1u;   // linked blocks (frames of one block: independent)
        const uint32_t flg = (1u << 6) | (indep << 5) | ((uint32_t)bcrc << 4) | ((uint32_t)csz << 3) | ((uint32_t)ccrc << 2);
        const uint32_t bd = (uint32_t)(bsid & 7) << 4;
        uint32_t hw[3] = {flg | (bd << 8), 0, 0};   // descriptor bytes as little-endian words
        int hl = 2;
        if (csz) {
            hw[0] |= (uint32_t)(s & 0xffff) << 16;
            hw[1] = (uint32_t)(s >> 16);
            hw[2] = (uint32_t)(s >> 48);
            hl = 10;
        }
        // XXH32 of the hl descriptor bytes (< 16: the short-input path, xxhash.c:383-388)
        uint32_t h = frm::P5 + (uint32_t)hl;
        int p = 0;
        for (; p + 4 <= hl; p += 4) h = frm::rotl(h + hw[p / 4] * frm::P3, 17) * frm::P4;
        for (; p < hl; p++) h = frm::rotl(h + ((hw[p / 4] >> (8 * (p & 3))) & 0xffu) * frm::P5, 11) * frm::P1;
        h ^= h >> 15; h *= frm::P2; h ^= h >> 13; h *= frm::P3; h ^= h >> 16;
        if (t == 0) {
            frm::put_le(dst, 0, 0x184D2204u, 4);
            for (int i = 0; i < hl; i++) dst.st8(4 + i, (hw[i / 4] >> (8 * (i & 3))) & 0xffu);
            dst.st8(4 + hl, (h >> 8) & 0xffu);
            frm::put_le(dst, (int)fsz - 4 - 4 * ccrc, 0, 4);   // end mark
        }
        if (ccrc) {   // content checksum of the frame's input (lz4frame.c:1005-1011)
            Bytes src;
            src.init(in + foff, min<uint64_t>(in_readable - foff, s + 16));
            const uint32_t c = frm::xxh32_wave(src, (uint32_t)s, t);
            if (t == 0) frm::put_le(dst, (int)fsz - 4, c, 4);
        }
    } else if (t == 0) {
        frm::put_le(dst, 0, 4, 8);                             // LZ4_FLAG
        frm::put_le(dst, 8, 32 + 8 * ((uint64_t)nb + 1), 8);   // metadata bytes
        frm::put_le(dst, 16, s, 8);                            // uncompressed size
        frm::put_le(dst, 24, (uint64_t)32768 << params, 8);    // chunk size (nvcomp's, also when the input is smaller)
        frm::put_le(dst, 32, 32 + 8 * ((uint64_t)nb + 1), 8);  // offsets[0]
        frm::put_le(dst, 32 + 8 * (int)nb, fsz, 8);            // offsets[k] = total
    }
}

// ------------------------------------------------------------------------------------ decoding
// Block descriptor for the block decoder: u64 source offset in packed, u64 destination offset,
// u32 stored size, u32 decoded size, u32 flags (1 = stored raw), u32 spare.
struct FrameDesc { uint64_t src, dst; uint32_t cs, ds, flags, pad; };

// one wave per frame: header checks and block walk (lz4frame.c:1150-1260 LZ4F_decodeHeader,
// :1384-1899 LZ4F_decompress; nvcomp: LZ4Metadata.cpp:60-110), descriptors for every block
// (maxbpf slots per frame, unused slots decode nothing), fstat[f] = 0 or a negative status:
// -1 malformed, -2 a feature outside the supported set (dictionary id, blocks that are not all full
// but the last).  A linked frame's blocks are marked so that one wave decodes them in order, each
// with the frame's output before it as its prefix (LZ4F_updateDict, lz4frame.c:1290-1306).
extern "C" __global__ void __launch_bounds__(64)
lzh_frame_parse_kernel(int codec, const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                       const uint32_t* csizes, uint64_t n_total, uint64_t fs, uint32_t maxbpf, FrameDesc* desc,
                       int32_t* fstat) {
    const int lane = threadIdx.x;
    const uint64_t f = blockIdx.x;
    const uint64_t foff = f * fs;
    if (foff >= n_total) return;
    const uint64_t s = min(fs, n_total - foff);
    const uint64_t ioff = offsets[f];
    const uint32_t cs = csizes[f];
    FrameDesc* D = desc + f * maxbpf;
    for (uint32_t b = (uint32_t)lane; b < maxbpf; b += 64) D[b] = FrameDesc{0, 0, 0, 0, 0, 0};
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");   // the zeroing before lane 0's descriptor stores
    __syncthreads();
    if (cs == s) {   // stored raw by the chunk loop (lzbench.cpp:318-321)
        if (lane == 0) { D[0] = FrameDesc{ioff, foff, cs, (uint32_t)s, 1, 0}; fstat[f] = 0; }
        return;
    }
    Bytes fr;
    const uint64_t readable = ioff < packed_readable ? min<uint64_t>(packed_readable - ioff, (uint64_t)cs + 16) : 0;
    fr.init(packed + ioff, readable);
    auto rd = [&](uint32_t p) -> uint32_t { return uni(fr.w32((int)p)); };
    int st = 0;
    if (codec == 4) {
        const uint32_t w0 = rd(0), w1 = rd(4);
        const uint32_t flg = w1 & 0xffu, bd = (w1 >> 8) & 0xffu;
        const int bcrc = (flg >> 4) & 1, csz = (flg >> 3) & 1, ccrc = (flg >> 2) & 1, dict = flg & 1;
        const uint32_t hl = 7 + 8 * csz + 4 * dict;
        const int bid = (int)(bd >> 4) & 7;
        if (cs < 7 || w0 != 0x184D2204u || (flg >> 6) != 1 || (flg & 2) || (bd & 0x8f) || bid < 4 || cs < hl) st = -1;
        if (!st) {   // header checksum over FLG .. the optional fields
            const uint32_t hcb = (rd(hl - 1) & 0xffu);
            const uint32_t hw[4] = {rd(4), rd(8), rd(12), rd(16)};   // bytes 4 .. hl - 2 (up to 17)
            const int n = (int)hl - 5;
            uint32_t h = frm::P5 + (uint32_t)n;
            int p = 0;
            for (; p + 4 <= n; p += 4) h = frm::rotl(h + hw[p / 4] * frm::P3, 17) * frm::P4;
            for (; p < n; p++) h = frm::rotl(h + ((hw[p / 4] >> (8 * (p & 3))) & 0xffu) * frm::P5, 11) * frm::P1;
            h ^= h >> 15; h *= frm::P2; h ^= h >> 13; h *= frm::P3; h ^= h >> 16;
            if (hcb != ((h >> 8) & 0xffu)) st = -1;
            else if (dict) st = -2;
            else if (csz && (((uint64_t)rd(10) << 32 | rd(6)) != s)) st = -1;
        }
        const uint64_t B = frm::bsize_of(bid);
        const uint32_t nbe = st ? 0 : (uint32_t)((s + B - 1) / B);   // blocks a full-block frame has
        uint32_t ip = hl, b = 0;
        while (!st) {
            if (ip + 4 > cs) { st = -1; break; }
            const uint32_t w = rd(ip);
            ip += 4;
            if (w == 0) break;
            const uint32_t sz = w & 0x7fffffffu;
            if (sz > B || ip + sz + 4u * (uint32_t)bcrc > cs) { st = -1; break; }
            if (b >= nbe) { st = -2; break; }
            const uint32_t ds = (uint32_t)min<uint64_t>(B, s - b * B);
            const bool raw = (w >> 31) != 0;
            if (raw && sz != ds) { st = sz > ds ? -1 : -2; break; }
            if (bcrc) {
                Bytes bb;
                bb.init_dw(packed + ioff + ip, min<uint64_t>(sz, readable > ip ? readable - ip : 0));
                const uint32_t h = frm::xxh32_wave(bb, sz, lane);
                if (h != rd(ip + sz)) { st = -1; break; }
            }
            // flags: 1 = stored raw, 2 = a linked frame's first block (pad = the frame's block count),
            // 4 = a linked frame's later block (decoded by the first block's wave, in order)
            const uint32_t lk = (flg & 0x20) ? 0u : (b == 0 ? 2u : 4u);
            if (lane == 0) D[b] = FrameDesc{ioff + ip, foff + b * B, sz, ds, (raw ? 1u : 0u) | lk, 0};
            ip += sz + 4u * (uint32_t)bcrc;
            b++;
        }
        if (!st && b != nbe) st = -2;
        if (!st && !(flg & 0x20) && lane == 0) D[0].pad = b;
        if (!st && ccrc) ip += 4;
        if (!st && ip != cs) st = -1;
    } else {
        const uint64_t flag = (uint64_t)rd(4) << 32 | rd(0), M = (uint64_t)rd(12) << 32 | rd(8);
        const uint64_t n = (uint64_t)rd(20) << 32 | rd(16), C = (uint64_t)rd(28) << 32 | rd(24);
        if (cs < 40 || flag != 4 || n != s) st = -1;
        else if (C < (32u << 10) || C > s * 0 + ((uint64_t)1 << 31)) st = -2;   // slots are sized for chunks >= 32 KiB
        const uint64_t k = st ? 0 : (n + C - 1) / C;
        if (!st && (M != (4 + k + 1) * 8 || M > cs)) st = -1;
        for (uint64_t b = 0; !st && b < k; b++) {
            const uint32_t p = 32 + 8 * (uint32_t)b;
            const uint64_t a = (uint64_t)rd(p + 4) << 32 | rd(p), e = (uint64_t)rd(p + 12) << 32 | rd(p + 8);
            if (a < M || e < a || e > cs) { st = -1; break; }
            if (lane == 0) D[b] = FrameDesc{ioff + a, foff + b * C, (uint32_t)(e - a), (uint32_t)min(C, n - b * C), 0, 0};
        }
    }
    if (lane == 0) fstat[f] = st;
}

// one wave per frame: the blocks' decoded sizes, the content checksum (lz4frame.c:1810-1830)
extern "C" __global__ void __launch_bounds__(64)
lzh_frame_finish_kernel(int codec, const uint8_t* packed, const uint64_t* offsets, const uint32_t* csizes,
                        uint64_t n_total, uint64_t fs, uint32_t maxbpf, const FrameDesc* desc, const int32_t* bstat,
                        const int32_t* fstat, const uint8_t* out, int32_t* status) {
    const int lane = threadIdx.x;
    const uint64_t f = blockIdx.x;
    const uint64_t foff = f * fs;
    if (foff >= n_total) return;
    const uint64_t s = min(fs, n_total - foff);
    int st = fstat[f];
    const FrameDesc* D = desc + f * maxbpf;
    for (uint32_t b0 = 0; !st && b0 < maxbpf; b0 += 64) {
        const uint32_t b = b0 + (uint32_t)lane;
        bool badb = false, shortb = false;
        if (b < maxbpf && D[b].ds) {
            const int r = bstat[f * maxbpf + b];
            badb = r < 0 || r > (int)D[b].ds;
            shortb = r >= 0 && r < (int)D[b].ds;
        }
        if (ballot(badb)) st = -1;
        else if (ballot(shortb)) st = -2;
    }
    if (!st && codec == 4 && csizes[f] != s) {
        Bytes fr;
        fr.init(packed + offsets[f], 8);
        const uint32_t flg = uni(fr.w32(4)) & 0xffu;
        if ((flg >> 2) & 1) {
            Bytes o, tail;
            o.init_dw(out + foff, s);
            const uint32_t h = frm::xxh32_wave(o, (uint32_t)s, lane);
            tail.init(packed + offsets[f] + csizes[f] - 4, 4);   // (bytewise: the range ends at the frame's end)
            const uint32_t c = tail.b(0) | tail.b(1) << 8 | tail.b(2) << 16 | tail.b(3) << 24;
            if (h != uni(c)) st = -1;
        }
    }
    if (lane == 0) status[f] = st ? st : (int32_t)s;
}

#include "launch.h"
hipError_t lzh_launch_frame_sizes(int codec, int params, uint64_t n_total, uint64_t fs, uint64_t bs, uint32_t bpf,
                                  const uint32_t* bcs, uint32_t* rel, uint32_t* csizes, uint32_t nframes, hipStream_t s) {
    if (!nframes) return hipSuccess;
    hipLaunchKernelGGL(lzh_frame_size_kernel, dim3((nframes + 255) / 256), dim3(256), 0, s, codec, params, n_total, fs,
                       bs, bpf, bcs, rel, csizes, nframes);
    return hipGetLastError();
}
hipError_t lzh_launch_frame_pack(int codec, int params, const uint8_t* in, uint64_t n_total, uint64_t in_readable,
                                 uint64_t fs, uint64_t bs, uint32_t bpf, const uint8_t* stage, uint64_t stride,
                                 const uint32_t* bcs, const uint32_t* rel, const uint32_t* csizes,
                                 const uint64_t* offsets, uint8_t* packed, uint32_t nblocks, uint32_t nframes,
                                 hipStream_t s) {
    if (!nframes) return hipSuccess;
    hipLaunchKernelGGL(lzh_frame_pack_kernel, dim3(nblocks + nframes), dim3(256), 0, s, codec, params, in, n_total,
                       in_readable, fs, bs, bpf, stage, stride, bcs, rel, csizes, offsets, packed, nblocks);
    return hipGetLastError();
}
hipError_t lzh_launch_frame_parse(int codec, const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                                  const uint32_t* csizes, uint64_t n_total, uint64_t fs, uint32_t maxbpf, void* desc,
                                  int32_t* fstat, uint32_t nframes, hipStream_t s) {
    if (!nframes) return hipSuccess;
    hipLaunchKernelGGL(lzh_frame_parse_kernel, dim3(nframes), dim3(64), 0, s, codec, packed, packed_readable, offsets,
                       csizes, n_total, fs, maxbpf, (FrameDesc*)desc, fstat);
    return hipGetLastError();
}
hipError_t lzh_launch_frame_finish(int codec, const uint8_t* packed, const uint64_t* offsets, const uint32_t* csizes,
                                   uint64_t n_total, uint64_t fs, uint32_t maxbpf, const void* desc,
                                   const int32_t* bstat, const int32_t* fstat, const uint8_t* out, int32_t* status,
                                   uint32_t nframes, hipStream_t s) {
    if (!nframes) return hipSuccess;
    hipLaunchKernelGGL(lzh_frame_finish_kernel, dim3(nframes), dim3(64), 0, s, codec, packed, offsets, csizes, n_total,
                       fs, maxbpf, (const FrameDesc*)desc, bstat, fstat, out, status);
    return hipGetLastError();
}
