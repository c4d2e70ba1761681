/*
 * oracle/ref_wrap.cpp -- extern "C" shims over the REFERENCE codecs, compiled straight from
 * /root/reference/lz4/lz4.c and /root/reference/snappy/*.cc by oracle/Makefile into
 * oracle/_ref/libref.so.  TEST INFRASTRUCTURE ONLY: used to pin the oracle restatement
 * (golden vectors) and as bench.py's cpu_baseline (kind "reference").  No reference source
 * is copied into this repository; this file only calls the reference's public API.
 *
 * The chunk loops mirror lzbench's exactly:
 *   lzbench_compress   /root/reference/_lzbench/lzbench.cpp:266-298
 *   lzbench_decompress /root/reference/_lzbench/lzbench.cpp:301-329
 *   lz4 row adapters   /root/reference/_lzbench/compressors.cpp:343-362
 *     (LZ4_compress_default / LZ4_compress_fast(level), LZ4_decompress_fast)
 *   snappy adapters    /root/reference/_lzbench/compressors.cpp:1282-1292
 *   zstd adapters      /root/reference/_lzbench/compressors.cpp:1745-1778 (codec 2: ZSTD_getParams(level,
 *                      part, 0), contentSizeFlag = 1, ZSTD_compress_advanced; ZSTD_decompressDCtx)
 *   codec 3            one LZ4 frame per chunk: LZ4F_compressFrame (lz4/lz4frame.c:429-470) with
 *                      independent or linked blocks and the requested block size / checksums /
 *                      content size;
 *                      LZ4F_decompress (lz4frame.c:1384) over the whole frame
 *   codec 4            one nvcomp LZ4 container per chunk (nvcomp/LZ4Metadata.h layout, restated as in
 *                      oracle/frame_oracle.c: nvcomp itself cannot be built) around reference
 *                      LZ4_compress_default blocks of 1 << (15 + level) bytes
 */
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <memory>
#include <thread>
#include <vector>
#include "lz4.h"
#include "lz4frame.h"
#include "snappy.h"
#define ZSTD_STATIC_LINKING_ONLY   /* ZSTD_compress_advanced, as lzbench uses it */
#include "zstd.h"

#define REF_COMPRESS_BOUND(n) ((n) + (n) / 6 + 16 * 1024)   /* GET_COMPRESS_BOUND, lzbench.h:17 */

extern "C" {

int ref_lz4_version(void) { return LZ4_versionNumber(); }
int ref_lz4_compress_fast(const char* s, char* d, int n, int cap, int acc) { return LZ4_compress_fast(s, d, n, cap, acc); }
int ref_lz4_compress_default(const char* s, char* d, int n, int cap) { return LZ4_compress_default(s, d, n, cap); }
int ref_lz4_decompress_safe(const char* s, char* d, int csize, int cap) { return LZ4_decompress_safe(s, d, csize, cap); }
int ref_lz4_decompress_fast(const char* s, char* d, int osize) { return LZ4_decompress_fast(s, d, osize); }
size_t ref_snappy_compress(const char* s, size_t n, char* d) { size_t out = 0; snappy::RawCompress(s, n, d, &out); return out; }
int ref_snappy_uncompress(const char* s, size_t csize, char* d) { return snappy::RawUncompress(s, csize, d) ? 1 : 0; }
size_t ref_snappy_max_compressed_length(size_t n) { return snappy::MaxCompressedLength(n); }

// one compression / decompression context per thread, created once (lzbench_zstd_init)
struct ZstdCtx {
    ZSTD_CCtx* c = ZSTD_createCCtx();
    ZSTD_DCtx* d = ZSTD_createDCtx();
    ~ZstdCtx() { ZSTD_freeCCtx(c); ZSTD_freeDCtx(d); }
};
static ZstdCtx& zctx() { static thread_local ZstdCtx z; return z; }

int64_t ref_zstd_compress(const char* in, size_t n, char* out, size_t cap, int level) {
    ZSTD_parameters p = ZSTD_getParams(level, n, 0);
    ZSTD_CCtx_setParameter(zctx().c, ZSTD_c_compressionLevel, level);
    p.fParams.contentSizeFlag = 1;
    const size_t r = ZSTD_compress_advanced(zctx().c, out, cap, in, n, NULL, 0, p);
    return ZSTD_isError(r) ? -1 : (int64_t)r;
}
/* the same frame with the XXH64 content checksum (fParams.checksumFlag), for the decoder's checksum path */
int64_t ref_zstd_compress_checksum(const char* in, size_t n, char* out, size_t cap, int level) {
    ZSTD_parameters p = ZSTD_getParams(level, n, 0);
    ZSTD_CCtx_setParameter(zctx().c, ZSTD_c_compressionLevel, level);
    p.fParams.contentSizeFlag = 1;
    p.fParams.checksumFlag = 1;
    const size_t r = ZSTD_compress_advanced(zctx().c, out, cap, in, n, NULL, 0, p);
    return ZSTD_isError(r) ? -1 : (int64_t)r;
}
int64_t ref_zstd_decompress(const char* in, size_t csize, char* out, size_t cap) {
    const size_t r = ZSTD_decompressDCtx(zctx().d, out, cap, in, csize);
    return ZSTD_isError(r) ? -1 : (int64_t)r;
}
int ref_zstd_version(void) { return (int)ZSTD_versionNumber(); }

/* params as oracle_lz4f_compress: bits 0-2 blockSizeID (0 default), 0x10 block checksum, 0x20 content
 * checksum, 0x40 content size, 0x80 linked blocks (LZ4F_blockLinked, the LZ4F default), bits 8-15
 * acceleration (compressionLevel = -(acc - 1)) */
static LZ4F_preferences_t lz4f_prefs(size_t n, int params) {
    LZ4F_preferences_t p;
    memset(&p, 0, sizeof(p));
    p.frameInfo.blockSizeID = (LZ4F_blockSizeID_t)(params & 7);
    p.frameInfo.blockMode = (params & 0x80) ? LZ4F_blockLinked : LZ4F_blockIndependent;
    p.frameInfo.blockChecksumFlag = (params & 0x10) ? LZ4F_blockChecksumEnabled : LZ4F_noBlockChecksum;
    p.frameInfo.contentChecksumFlag = (params & 0x20) ? LZ4F_contentChecksumEnabled : LZ4F_noContentChecksum;
    p.frameInfo.contentSize = (params & 0x40) ? (unsigned long long)n : 0;
    const int acc = (params >> 8) & 0xff;
    p.compressionLevel = acc > 1 ? -(acc - 1) : 0;
    return p;
}
size_t ref_lz4f_bound(size_t n, int params) {
    LZ4F_preferences_t p = lz4f_prefs(n, params);
    return LZ4F_compressFrameBound(n, &p);
}
int64_t ref_lz4f_compress(const char* in, size_t n, char* out, size_t cap, int params) {
    LZ4F_preferences_t p = lz4f_prefs(n, params);
    const size_t r = LZ4F_compressFrame(out, cap, in, n, &p);
    return LZ4F_isError(r) ? -1 : (int64_t)r;
}
/* whole frame -> decoded size, -1 on any LZ4F error or a frame that does not end exactly at csize */
int64_t ref_lz4f_decompress(const char* in, size_t csize, char* out, size_t cap) {
    LZ4F_dctx* d = nullptr;
    if (LZ4F_isError(LZ4F_createDecompressionContext(&d, LZ4F_VERSION))) return -1;
    size_t ip = 0, op = 0;
    int64_t res = -1;
    for (;;) {
        size_t isz = csize - ip, osz = cap - op;
        const size_t r = LZ4F_decompress(d, out + op, &osz, in + ip, &isz, nullptr);
        if (LZ4F_isError(r)) break;
        ip += isz;
        op += osz;
        if (r == 0) { res = ip == csize ? (int64_t)op : -1; break; }
        if (isz == 0 && osz == 0) break;   /* needs input it does not have: truncated */
    }
    LZ4F_freeDecompressionContext(d);
    return res;
}

static void put64(char* p, uint64_t v) { memcpy(p, &v, 8); }   /* (x86: little endian) */
int64_t ref_nvlz4_compress(const char* in, size_t n, char* out, size_t cap, int level) {
    const size_t C = (size_t)1 << (15 + level), k = (n + C - 1) / C;
    const uint64_t M = (4 + k + 1) * 8;
    if (cap < M) return -1;
    put64(out, 4); put64(out + 8, M); put64(out + 16, n); put64(out + 24, C);
    uint64_t off = M;
    for (size_t i = 0; i < k; i++) {
        put64(out + 32 + 8 * i, off);
        const int bs = (int)std::min(C, n - i * C);
        const int r = LZ4_compress_default(in + i * C, out + off, bs, (int)(cap - off));
        if (r <= 0) return -1;
        off += (uint64_t)r;
    }
    put64(out + 32 + 8 * k, off);
    return (int64_t)off;
}
int64_t ref_nvlz4_decompress(const char* in, size_t csize, char* out, size_t cap) {
    uint64_t h[4];
    if (csize < 40) return -1;
    memcpy(h, in, 32);
    if (h[0] != 4 || h[3] == 0 || h[2] > cap) return -1;
    const uint64_t k = (h[2] + h[3] - 1) / h[3];
    if (h[1] != (4 + k + 1) * 8 || h[1] > csize) return -1;
    for (uint64_t i = 0; i < k; i++) {
        uint64_t a, b;
        memcpy(&a, in + 32 + 8 * i, 8);
        memcpy(&b, in + 40 + 8 * i, 8);
        const int bs = (int)std::min<uint64_t>(h[3], h[2] - i * h[3]);
        if (a < h[1] || b < a || b > csize) return -1;
        if (LZ4_decompress_safe(in + a, out + i * h[3], (int)(b - a), bs) != bs) return -1;
    }
    return (int64_t)h[2];
}

static int64_t one_compress(int codec, int level, const char* in, size_t part, char* out, size_t outpart) {
    if (codec == 3) { const int64_t r = ref_lz4f_compress(in, part, out, outpart, level); return r < 0 ? 0 : r; }
    if (codec == 4) { const int64_t r = ref_nvlz4_compress(in, part, out, outpart, level); return r < 0 ? 0 : r; }
    if (codec == 2) {
        const int64_t r = ref_zstd_compress(in, part, out, outpart, level);   /* zstd_fast rows pass -5..-1 */
        return r < 0 ? 0 : r;
    }
    if (codec == 0) {
        if (level <= 1) return LZ4_compress_default(in, out, (int)part, (int)outpart);
        return LZ4_compress_fast(in, out, (int)part, (int)outpart, level);
    }
    size_t o = outpart;
    snappy::RawCompress(in, part, out, &o);
    return (int64_t)o;
}

static int64_t one_decompress(int codec, const char* in, size_t csize, char* out, size_t osize) {
    if (codec == 2) return ref_zstd_decompress(in, csize, out, osize);
    if (codec == 3) return ref_lz4f_decompress(in, csize, out, osize);
    if (codec == 4) return ref_nvlz4_decompress(in, csize, out, osize);
    if (codec == 0) { LZ4_decompress_fast(in, out, (int)osize); return (int64_t)osize; }
    snappy::RawUncompress(in, csize, out);
    return (int64_t)osize;
}

/* lzbench_compress over [c0,c1): packs into out, returns bytes */
static int64_t range_compress(int codec, int level, const uint8_t* in, size_t n, size_t chunk,
                              size_t c0, size_t c1, uint8_t* out, size_t outsize, uint64_t* csizes) {
    size_t nchunks = (n + chunk - 1) / chunk;
    int64_t sum = 0;
    for (size_t i = c0; i < c1; i++) {
        size_t part = (i + 1 < nchunks) ? chunk : n - i * chunk;
        size_t outpart = REF_COMPRESS_BOUND(part);
        if (outpart > outsize) outpart = outsize;
        const uint8_t* src = in + i * chunk;
        int64_t clen = one_compress(codec, level, (const char*)src, part, (char*)out, outpart);
        if (clen <= 0 || (size_t)clen == part) {
            if (part > outsize) return 0;
            memcpy(out, src, part);
            clen = (int64_t)part;
        }
        out += clen; outsize -= (size_t)clen; csizes[i] = (uint64_t)clen; sum += clen;
    }
    return sum;
}

int64_t ref_compress_chunks(int codec, int level, const uint8_t* in, size_t n, size_t chunk,
                            uint8_t* out, uint64_t* csizes) {
    size_t nchunks = (n + chunk - 1) / chunk;
    return range_compress(codec, level, in, n, chunk, 0, nchunks, out, REF_COMPRESS_BOUND(n), csizes);
}

int64_t ref_decompress_chunks(int codec, const uint8_t* packed, const uint64_t* csizes, size_t n,
                              size_t chunk, uint8_t* out) {
    size_t nchunks = (n + chunk - 1) / chunk;
    int64_t sum = 0;
    for (size_t i = 0; i < nchunks; i++) {
        size_t part = (i + 1 < nchunks) ? chunk : n - i * chunk;
        int64_t d;
        if (csizes[i] == part) { memcpy(out, packed, part); d = (int64_t)part; }
        else d = one_decompress(codec, (const char*)packed, csizes[i], (char*)out, part);
        if (d <= 0) return d;
        packed += csizes[i]; out += d; sum += d;
    }
    return sum;
}

/* all-cores variants: contiguous chunk ranges per thread, private staging, ordered gather */
int64_t ref_compress_chunks_mt(int codec, int level, const uint8_t* in, size_t n, size_t chunk,
                               uint8_t* out, uint64_t* csizes, int threads) {
    size_t nchunks = (n + chunk - 1) / chunk;
    if (threads < 1) threads = 1;
    if ((size_t)threads > nchunks) threads = nchunks ? (int)nchunks : 1;
    std::vector<std::unique_ptr<uint8_t[]>> stage((size_t)threads);
    std::vector<size_t> stage_cap((size_t)threads);
    std::vector<int64_t> res((size_t)threads, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        size_t c0 = nchunks * (size_t)t / (size_t)threads, c1 = nchunks * (size_t)(t + 1) / (size_t)threads;
        size_t span = (c1 - c0) * chunk;
        stage_cap[(size_t)t] = REF_COMPRESS_BOUND(span) + 64;
        stage[(size_t)t].reset(new uint8_t[stage_cap[(size_t)t]]);   /* no zero fill */
        th.emplace_back([&, t, c0, c1]() {
            res[(size_t)t] = range_compress(codec, level, in, n, chunk, c0, c1, stage[(size_t)t].get(),
                                            stage_cap[(size_t)t], csizes);
        });
    }
    int64_t sum = 0;
    for (int t = 0; t < threads; t++) {
        th[(size_t)t].join();
        memcpy(out + sum, stage[(size_t)t].get(), (size_t)res[(size_t)t]);
        sum += res[(size_t)t];
    }
    return sum;
}

int64_t ref_decompress_chunks_mt(int codec, const uint8_t* packed, const uint64_t* csizes, size_t n,
                                 size_t chunk, uint8_t* out, int threads) {
    size_t nchunks = (n + chunk - 1) / chunk;
    if (threads < 1) threads = 1;
    if ((size_t)threads > nchunks) threads = nchunks ? (int)nchunks : 1;
    std::vector<uint64_t> off(nchunks + 1, 0);
    for (size_t i = 0; i < nchunks; i++) off[i + 1] = off[i] + csizes[i];
    std::vector<int64_t> res((size_t)threads, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < threads; t++) {
        size_t c0 = nchunks * (size_t)t / (size_t)threads, c1 = nchunks * (size_t)(t + 1) / (size_t)threads;
        th.emplace_back([&, t, c0, c1]() {
            int64_t s = 0;
            for (size_t i = c0; i < c1; i++) {
                size_t part = (i + 1 < nchunks) ? chunk : n - i * chunk;
                int64_t d;
                if (csizes[i] == part) { memcpy(out + i * chunk, packed + off[i], part); d = (int64_t)part; }
                else d = one_decompress(codec, (const char*)packed + off[i], csizes[i], (char*)out + i * chunk, part);
                if (d <= 0) { s = d; break; }
                s += d;
            }
            res[(size_t)t] = s;
        });
    }
    int64_t sum = 0;
    for (int t = 0; t < threads; t++) { th[(size_t)t].join(); if (res[(size_t)t] <= 0) return -1; sum += res[(size_t)t]; }
    return sum;
}

}  // extern "C"
