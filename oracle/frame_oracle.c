/*
 * oracle/frame_oracle.c -- the framed LZ4 formats restated in C.  TEST INFRASTRUCTURE ONLY.
 *
 * 1. LZ4 frame (lz4frame.c 1.9.3) as LZ4F_compressFrame writes it, blocks independent or linked:
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
 *    Linked blocks (LZ4F_blockLinked, the LZ4F default; params flag 0x80): LZ4F_compressBegin resets
 *    the stream once per frame (lz4frame.c:651-655, LZ4F_initStream -> LZ4_resetStream_fast), and every
 *    block goes through LZ4F_compressBlock_continue -> LZ4_compress_fast_continue (lz4frame.c:777-782,
 *    lz4.c:1565-1628).  The blocks lie back to back in the caller's buffer (stableSrc), so each one is
 *    compressed in prefix mode: LZ4_compress_generic with byU32 / hash5, withPrefix64k, noDictIssue and
 *    limitedOutput (lz4.c:851-1240): positions are frame indices (base = the frame start, the table
 *    persists from block to block), candidates reach up to 65535 bytes back into earlier blocks, the
 *    catch-up stops at the frame start (lowLimit = source - dictSize), and a block that does not fit
 *    size - 1 bytes returns 0 where the first check fails (lz4.c:1024-1027, :1097-1121, :1207-1216),
 *    leaving the table as it stands there for the next block (restated inline: lz4f_linked_block).
 *    Decoding restates LZ4F_decompress (lz4frame.c:1384-1899) for one whole frame; a linked block
 *    decodes with everything decoded before it in the frame as its prefix (LZ4F_updateDict's prefix
 *    mode, lz4frame.c:1290-1306, and LZ4_decompress_safe_usingDict, lz4.c:2404-2416).
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

static uint32_t lz4f_h5(const uint8_t* p) {   /* LZ4_hash5 for byU32 (lz4.c:706-722) */
    const uint64_t v = (uint64_t)rd32(p) | (uint64_t)rd32(p + 4) << 32;
    return (uint32_t)(((v << 24) * 889523592379ull) >> 52);
}

static int lz4f_put_len(uint8_t* dst, int op, int len) {
    while (len >= 255) { dst[op++] = 255; len -= 255; }
    dst[op++] = (uint8_t)len;
    return op;
}

/* One block of a linked frame: f = the frame, the block = [b0, b0 + n), t = the frame's table
 * (4096 u32 indices, zeroed at the frame start).  LZ4_compress_generic's prefix-mode parse with the
 * limitedOutput checks at their places (olimit = cap = n - 1); returns the block size or 0. */
static int lz4f_linked_block(uint32_t* t, const uint8_t* f, int b0, int n, uint8_t* dst, int acc) {
    const int cap = n - 1, iend = b0 + n, mfl1 = iend - 12 + 1, mlimit = iend - 5;
    int ip = b0, anchor = b0, op = 0;
    uint32_t fh;
    if (n < 13) goto last_literals;                       /* lz4.c:921 */
    t[lz4f_h5(f + b0)] = (uint32_t)b0;                    /* first byte (lz4.c:924-925) */
    ip = b0 + 1;
    fh = lz4f_h5(f + ip);
    for (;;) {
        int match, tok;
        {   /* probe loop (lz4.c:954-1014) */
            int fwd = ip, step = 1, nb = acc << 6;
            for (;;) {
                const uint32_t h = fh;
                const int cur = fwd;
                const uint32_t cand = t[h];
                ip = fwd;
                fwd += step;
                step = nb++ >> 6;
                if (fwd > mfl1) goto last_literals;
                fh = lz4f_h5(f + fwd);
                t[h] = (uint32_t)cur;
                if (cand + 65535u < (uint32_t)cur) continue;             /* too far (lz4.c:1003) */
                if (rd32(f + cand) == rd32(f + ip)) { match = (int)cand; break; }
            }
        }
        /* catch up, down to the frame start (lowLimit = source - dictSize, lz4.c:1019) */
        while (ip > anchor && match > 0 && f[ip - 1] == f[match - 1]) { ip--; match--; }
        {   /* literals, with the limitedOutput check (lz4.c:1024-1027) */
            const int lit = ip - anchor;
            tok = op++;
            if (op + lit + 8 + lit / 255 > cap) return 0;
            if (lit >= 15) { dst[tok] = 15 << 4; op = lz4f_put_len(dst, op, lit - 15); }
            else dst[tok] = (uint8_t)(lit << 4);
            memcpy(dst + op, f + anchor, (size_t)lit);
            op += lit;
        }
    next_match:
        {
            const int off = ip - match;
            dst[op++] = (uint8_t)(off & 0xff);
            dst[op++] = (uint8_t)(off >> 8);
            int ml = 0;                                                  /* LZ4_count to matchlimit */
            while (ip + 4 + ml < mlimit && f[ip + 4 + ml] == f[match + 4 + ml]) ml++;
            ip += ml + 4;
            if (op + 6 + (ml + 240) / 255 > cap) return 0;              /* lz4.c:1097-1121 */
            if (ml >= 15) { dst[tok] = (uint8_t)(dst[tok] + 15); op = lz4f_put_len(dst, op, ml - 15); }
            else dst[tok] = (uint8_t)(dst[tok] + ml);
        }
        anchor = ip;
        if (ip >= mfl1) break;                                           /* lz4.c:1142 */
        t[lz4f_h5(f + ip - 2)] = (uint32_t)(ip - 2);                     /* lz4.c:1146 */
        {   /* immediate re-test (lz4.c:1159-1196): no literal check on this path */
            const uint32_t h = lz4f_h5(f + ip), cand = t[h];
            t[h] = (uint32_t)ip;
            if (cand + 65535u >= (uint32_t)ip && rd32(f + cand) == rd32(f + ip)) {
                match = (int)cand;
                tok = op++;
                dst[tok] = 0;
                goto next_match;
            }
        }
        ip++;
        fh = lz4f_h5(f + ip);
    }
last_literals:
    {   /* lz4.c:1204-1231 */
        const int run = iend - anchor;
        if (op + run + 1 + (run + 240) / 255 > cap) return 0;
        if (run >= 15) { dst[op++] = 15 << 4; op = lz4f_put_len(dst, op, run - 15); }
        else dst[op++] = (uint8_t)(run << 4);
        memcpy(dst + op, f + anchor, (size_t)run);
        op += run;
    }
    return op;
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
    /* a frame of one block is independent whatever was asked (lz4frame.c:394-395) */
    const int linked = (params & 0x80) && n > B;
    uint8_t* o = dst;
    wr32(o, 0x184D2204u);
    o += 4;
    uint8_t* hs = o;
    *o++ = (uint8_t)((1 << 6) | ((!linked) << 5) | (bcrc << 4) | (csz << 3) | (ccrc << 2));
    *o++ = (uint8_t)((bsid & 7) << 4);
    if (csz) { wr64(o, (uint64_t)n); o += 8; }
    *o = (uint8_t)((oracle_xxh32(hs, (size_t)(o - hs), 0) >> 8) & 0xff);
    o++;
    uint8_t* tmp = (uint8_t*)malloc((size_t)oracle_lz4_bound((int)B) + 64);
    uint32_t* tab = linked ? (uint32_t*)calloc(4096, sizeof(uint32_t)) : NULL;
    for (size_t p = 0; p < n; p += B) {
        const int bs = (int)(n - p < B ? n - p : B);
        int c, raw;
        if (linked) {
            c = lz4f_linked_block(tab, src, (int)p, bs, tmp, acc < 1 ? 1 : acc);
            raw = c == 0;
        } else {
            c = oracle_lz4_compress(src + p, bs, tmp, acc < 1 ? 1 : acc);
            raw = limited_fails(tmp, c, bs - 1);
        }
        uint32_t cs;
        if (raw) {
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
    free(tab);
    wr32(o, 0);
    o += 4;
    if (ccrc) { wr32(o, oracle_xxh32(src, n, 0)); o += 4; }
    return (int64_t)(o - dst);
}

/* LZ4F_decompress over one whole frame (lz4frame.c:1384-1899: header decode :1150-1260 with its
 * checks, block loop, block / content checksums); returns the decoded size, -1 on malformed input,
 * -2 for a dictionary id (not restated; the GPU decoder refuses it too).  A linked frame's blocks
 * decode with the frame's output so far as their prefix. */
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
        const uint32_t sz = w & 0x7fffffffu;
        if (sz > B || ip + sz + 4u * (uint32_t)bcrc > cs) return -1;
        if (bcrc && rd32(src + ip + sz) != oracle_xxh32(src + ip, sz, 0)) return -1;
        if (w >> 31) {
            if (op + sz > cap) return -1;
            memcpy(dst + op, src + ip, sz);
            op += sz;
        } else {
            const size_t room = cap - op < B ? cap - op : B;
            /* linked: LZ4_decompress_safe_usingDict with the prefix dst[0, op) (withPrefix64k from the
             * second block on, every earlier block being full: no offset reaches past it) */
            const int d = (flg & 0x20) ? oracle_lz4_decompress_safe(src + ip, (int)sz, dst + op, (int)room)
                                       : oracle_lz4_decompress_prefix(src + ip, (int)sz, dst + op, (int)room, (int64_t)op);
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
