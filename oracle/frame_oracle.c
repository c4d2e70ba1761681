/*
 * oracle/frame_oracle.c -- the framed LZ4 formats restated in C.  TEST INFRASTRUCTURE ONLY.
 *
 * 1. LZ4 frame (lz4frame.c 1.9.3) as LZ4F_compressFrame writes it with independent blocks:
 *      LZ4F_compressFrame_usingCDict  /root/reference/lz4/lz4frame.c:373-419 (optimal block size,
 *                                     autoFlush, single-block frames independent)
 *      LZ4F_optimalBSID               lz4frame.c:304-316
 *      LZ4F_compressBegin_usingCDict  lz4frame.c:598-700 (magic, FLG, BD, content size, HC byte)
 *      LZ4F_makeBlock                 lz4frame.c:740-763 (dstCapacity = srcSize - 1, raw on failure,
 *                                     optional block checksum of the stored bytes)
 *      LZ4F_compressBlock             lz4frame.c:766-775 -> LZ4_compress_fast_extState_fastReset
 *                                     (lz4.c:1316-1351: limitedOutput; every block >= 4 KiB, or the
 *                                     first of a frame, starts from a cleared table, lz4.c:806-843)
 *      LZ4F_compressUpdate / _End     lz4frame.c:825-927, :986-1019 (full blocks, the remainder,
 *                                     end mark, optional content checksum)
 *    A block's limitedOutput outcome (lz4.c:1024-1027, :1097-1121, :1207-1216) depends only on the
 *    sequence layout, because the parse does not: the notLimited block is produced and its tokens
 *    are walked with the same conditions (the match-length check at every sequence implies the
 *    literal check, so it and the last-literals check decide).
 *    Decoding restates LZ4F_decompress (lz4frame.c:1384-1899) for one whole frame.
 * 2. The nvcomp LZ4 container (nvcomp 1.2.2, the reference's nvcomp_lz4 row): 8-byte fields
 *      [LZ4_FLAG = 4, metadata bytes M = (4 + k + 1) * 8, uncompressed size, chunk size,
 *       offsets[0..k]] (nvcomp/LZ4Metadata.h:39-60, MutableLZ4MetadataOnGPU.cpp copyToGPU,
 *      LZ4MetadataOnGPU.cpp:42-46), offsets exclusive prefix sums of the chunk streams starting at
 *      M (LZ4CompressionKernels.cu:1038-1073), chunk streams back to back (copyToContig :1075-1097).
 *      Chunks of 1 << (15 + level) bytes (compressors.cpp:1863); every chunk an LZ4 block, never
 *      stored raw.  nvcomp cannot be built here, so the layout is "parity unpinned" beyond this
 *      restatement; the blocks inside are LZ4_compress_default blocks (pinned like every LZ4 block).
 * XXH32 restates /root/reference/lz4/xxhash.c:269-389.
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- XXH32 (xxhash.c:263-389) */
#define P1 2654435761U
#define P2 2246822519U
#define P3 3266489917U
#define P4 668265263U
#define P5 374761393U
static uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint32_t rd32(const uint8_t* p) { return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24; }
static void wr32(uint8_t* p, uint32_t v) { p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24); }
static void wr64(uint8_t* p, uint64_t v) { wr32(p, (uint32_t)v); wr32(p + 4, (uint32_t)(v >> 32)); }

uint32_t oracle_xxh32(const uint8_t* p, size_t len, uint32_t seed) {
    const uint8_t* e = p + len;
    uint32_t h;
    if (len >= 16) {
        uint32_t v[4] = {seed + P1 + P2, seed + P2, seed, seed - P1};
        do {   /* four lanes, one 4-byte word each per 16-byte stripe */
            for (int k = 0; k < 4; k++, p += 4) v[k] = rotl32(v[k] + rd32(p) * P2, 13) * P1;
        } while (p < e - 15);
        h = rotl32(v[0], 1) + rotl32(v[1], 7) + rotl32(v[2], 12) + rotl32(v[3], 18);
    } else {
        h = seed + P5;
    }
    h += (uint32_t)len;
    for (; p + 4 <= e; p += 4) h = rotl32(h + rd32(p) * P3, 17) * P4;
    for (; p < e; p++) h = rotl32(h + (uint32_t)*p * P5, 11) * P1;
    h ^= h >> 15; h *= P2; h ^= h >> 13; h *= P3; h ^= h >> 16;
    return h;
}

/* ---------------------------------------------------------------- LZ4 frame */
static size_t bsid_size(int id) { return (size_t)1 << (8 + 2 * id); }   /* LZ4F_getBlockSize: 4..7 */

/* LZ4F_optimalBSID (lz4frame.c:304-316), with 0 = LZ4F_default -> max64KB (lz4frame.c:640-641) */
static int optimal_bsid(int req, size_t n) {
    int id = 4;
    size_t mb = 64 << 10;
    while (req > id) {
        if (n <= mb) return id;
        id++;
        mb <<= 2;
    }
    return req ? req : 4;
}

/* would LZ4_compress_generic in limitedOutput mode with olimit = cap have returned 0 for the
 * block `blk` (lz4.c:1097-1121 per sequence, :1207-1216 for the last literals)? */
static int limited_fails(const uint8_t* blk, int bs, int cap) {
    int ip = 0;
    while (ip < bs) {
        const int pos = ip;
        const uint32_t tok = blk[ip++];
        int lit = (int)(tok >> 4), lx = 0;
        if (lit == 15) { uint32_t s; do { s = blk[ip++]; lit += (int)s; lx++; } while (s == 255); }
        ip += lit;
        if (ip >= bs) return pos + lit + 1 + (lit + 240) / 255 > cap;   /* last literals */
        ip += 2;
        int mc = (int)(tok & 15u);
        if (mc == 15) { uint32_t s; do { s = blk[ip++]; mc += (int)s; } while (s == 255); }
        if (pos + 1 + lx + lit + 2 + 6 + (mc + 240) / 255 > cap) return 1;
    }
    return 0;
}

size_t oracle_lz4f_bound(size_t n, int params) {
    const size_t B = bsid_size(optimal_bsid(params & 7, n));
    const size_t nb = (n + B - 1) / B;
    return 19 + nb * (4 + 4 + B) + 4 + 4 + 64;   /* maxFHSize + per block header/crc + end + checksum */
}

int64_t oracle_lz4f_compress(const uint8_t* src, size_t n, uint8_t* dst, int params) {
    const int bsid = optimal_bsid(params & 7, n);
    const int bcrc = (params & 0x10) != 0, ccrc = (params & 0x20) != 0, csz = (params & 0x40) && n > 0;
    const int acc = (params >> 8) & 0xff;
    const size_t B = bsid_size(bsid);
    uint8_t* o = dst;
    wr32(o, 0x184D2204u);
    o += 4;
    uint8_t* hs = o;
    *o++ = (uint8_t)((1 << 6) | (1 << 5) | (bcrc << 4) | (csz << 3) | (ccrc << 2));
    *o++ = (uint8_t)((bsid & 7) << 4);
    if (csz) { wr64(o, (uint64_t)n); o += 8; }
    *o = (uint8_t)((oracle_xxh32(hs, (size_t)(o - hs), 0) >> 8) & 0xff);
    o++;
    uint8_t* tmp = (uint8_t*)malloc((size_t)oracle_lz4_bound((int)B) + 64);
    for (size_t p = 0; p < n; p += B) {
        const int bs = (int)(n - p < B ? n - p : B);
        const int c = oracle_lz4_compress(src + p, bs, tmp, acc < 1 ? 1 : acc);
        uint32_t cs;
        if (limited_fails(tmp, c, bs - 1)) {
            cs = (uint32_t)bs;
            wr32(o, cs | 0x80000000u);
            memcpy(o + 4, src + p, (size_t)bs);
        } else {
            cs = (uint32_t)c;
            wr32(o, cs);
            memcpy(o + 4, tmp, (size_t)c);
        }
        if (bcrc) wr32(o + 4 + cs, oracle_xxh32(o + 4, cs, 0));
        o += 4 + cs + 4 * bcrc;
    }
    free(tmp);
    wr32(o, 0);
    o += 4;
    if (ccrc) { wr32(o, oracle_xxh32(src, n, 0)); o += 4; }
    return (int64_t)(o - dst);
}

/* LZ4F_decompress over one whole frame (lz4frame.c:1384-1899: header decode :1150-1260 with its
 * checks, block loop, block / content checksums); returns the decoded size, -1 on malformed input,
 * -2 for a dictionary id or a second linked block (not restated; the GPU decoder refuses them too) */
int64_t oracle_lz4f_decompress(const uint8_t* src, size_t cs, uint8_t* dst, size_t cap) {
    if (cs < 7 || rd32(src) != 0x184D2204u) return -1;
    const uint32_t flg = src[4], bd = src[5];
    if ((flg >> 6) != 1 || (flg & 2) || (bd & 0x8f)) return -1;
    const int bid = (int)(bd >> 4) & 7;
    if (bid < 4) return -1;
    const int bcrc = (flg >> 4) & 1, csz = (flg >> 3) & 1, ccrc = (flg >> 2) & 1, dict = flg & 1;
    const size_t hl = 7 + 8 * (size_t)csz + 4 * (size_t)dict;
    if (cs < hl) return -1;
    /* LZ4F_decodeHeader's order (lz4frame.c:1150-1260): the header checksum, then the dictionary id */
    if (src[hl - 1] != (uint8_t)((oracle_xxh32(src + 4, hl - 5, 0) >> 8) & 0xff)) return -1;
    if (dict) return -2;
    const size_t B = bsid_size(bid);
    size_t ip = hl, op = 0;
    for (int nb = 0;; nb++) {
        if (ip + 4 > cs) return -1;
        const uint32_t w = rd32(src + ip);
        ip += 4;
        if (w == 0) break;
        if (nb > 0 && !(flg & 0x20)) return -2;   /* linked blocks past the first: not restated */
        const uint32_t sz = w & 0x7fffffffu;
        if (sz > B || ip + sz + 4u * (uint32_t)bcrc > cs) return -1;
        if (bcrc && rd32(src + ip + sz) != oracle_xxh32(src + ip, sz, 0)) return -1;
        if (w >> 31) {
            if (op + sz > cap) return -1;
            memcpy(dst + op, src + ip, sz);
            op += sz;
        } else {
            const size_t room = cap - op < B ? cap - op : B;
            const int d = oracle_lz4_decompress_safe(src + ip, (int)sz, dst + op, (int)room);
            if (d < 0) return -1;
            op += (size_t)d;
        }
        ip += sz + 4u * (uint32_t)bcrc;
    }
    if (ccrc) {
        if (ip + 4 > cs || rd32(src + ip) != oracle_xxh32(dst, op, 0)) return -1;
        ip += 4;
    }
    if (ip != cs) return -1;   /* a chunk is exactly one frame */
    if (csz) {
        const uint64_t c = (uint64_t)rd32(src + 6) | (uint64_t)rd32(src + 10) << 32;
        if (c != op) return -1;
    }
    return (int64_t)op;
}

/* ---------------------------------------------------------------- nvcomp LZ4 container */
size_t oracle_nvlz4_bound(size_t n, int level) {
    const size_t C = (size_t)1 << (15 + level), k = (n + C - 1) / C;
    return 32 + 8 * (k + 1) + k * (size_t)oracle_lz4_bound((int)C) + 64;
}

int64_t oracle_nvlz4_compress(const uint8_t* src, size_t n, uint8_t* dst, int level) {
    const size_t C = (size_t)1 << (15 + level), k = (n + C - 1) / C;
    const uint64_t M = (4 + k + 1) * 8;
    wr64(dst, 4); wr64(dst + 8, M); wr64(dst + 16, n); wr64(dst + 24, C);
    uint64_t off = M;
    for (size_t i = 0; i < k; i++) {
        wr64(dst + 32 + 8 * i, off);
        const int bs = (int)(n - i * C < C ? n - i * C : C);
        off += (uint64_t)oracle_lz4_compress(src + i * C, bs, dst + off, 1);
    }
    wr64(dst + 32 + 8 * k, off);
    return (int64_t)off;
}

int64_t oracle_nvlz4_decompress(const uint8_t* src, size_t cs, uint8_t* dst, size_t cap) {
    if (cs < 40) return -1;
    const uint64_t flag = rd32(src) | (uint64_t)rd32(src + 4) << 32;
    const uint64_t M = rd32(src + 8) | (uint64_t)rd32(src + 12) << 32;
    const uint64_t n = rd32(src + 16) | (uint64_t)rd32(src + 20) << 32;
    const uint64_t C = rd32(src + 24) | (uint64_t)rd32(src + 28) << 32;
    if (flag != 4 || C == 0 || n > cap) return -1;
    const uint64_t k = (n + C - 1) / C;
    if (M != (4 + k + 1) * 8 || M > cs) return -1;
    for (uint64_t i = 0; i < k; i++) {
        const uint8_t* q = src + 32 + 8 * i;
        const uint64_t a = rd32(q) | (uint64_t)rd32(q + 4) << 32, b = rd32(q + 8) | (uint64_t)rd32(q + 12) << 32;
        const uint64_t bs = n - i * C < C ? n - i * C : C;
        if (a < M || b < a || b > cs) return -1;
        if (oracle_lz4_decompress_safe(src + a, (int)(b - a), dst + i * C, (int)bs) != (int)bs) return -1;
    }
    return (int64_t)n;
}
