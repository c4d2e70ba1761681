/*
 * oracle/zstd1_oracle.c -- zstd 1.5.2 frame compression with the "fast" strategy (lzbench's
 * zstd row at level 1 and 2, zstd_fast at -1..-5) restated in plain C.  TEST INFRASTRUCTURE ONLY.
 *
 * What lzbench calls (/root/reference/_lzbench/compressors.cpp:1745-1770):
 *   p = ZSTD_getParams(level, part, 0); p.fParams.contentSizeFlag = 1;
 *   ZSTD_compress_advanced(cctx, out, outsize, in, part, NULL, 0, p)
 * Reference call chain (all under /root/reference/zstd/lib/):
 *   parameters      compress/zstd_compress.c:6272-6300 (ZSTD_getCParams_internal, tableID rule),
 *                   :1316-1373 (ZSTD_adjustCParams_internal), compress/clevels.h:25-130
 *   frame           zstd_compress.c:4111-4170 (ZSTD_compressContinue_internal), :4012-4058 (header),
 *                   :3932-4009 (ZSTD_compress_frameChunk: blocks of min(128 KiB, 2^windowLog))
 *   block           zstd_compress.c:3762-3824 (ZSTD_compressBlock_internal: raw / RLE / compressed,
 *                   repcodes + entropy tables confirmed only for compressed blocks), :2814-2893
 *   match finder    compress/zstd_fast.c:92-315 (ZSTD_compressBlock_fast_noDict_generic)
 *   entropy         zstd_compress.c:2573-2719 (ZSTD_entropyCompressSeqStore{,_internal}),
 *                   :2451-2566 (ZSTD_buildSequencesStatistics), :2388-2408 (ZSTD_seqToCodes)
 *   literals        compress/zstd_compress_literals.c:16-159, compress/huf_compress.c
 *                   (HUF_compress_internal :1177-1282, tree :308-708, table header :92-208,
 *                   stream :766-1130)
 *   FSE             compress/fse_compress.c (FSE_buildCTable_wksp :67-213, FSE_writeNCount :232-338,
 *                   FSE_optimalTableLog :356-382, FSE_normalizeCount :387-533, FSE compress :593-662),
 *                   compress/zstd_compress_sequences.c:157-382 (type selection, CTable build, encoder)
 *   histograms      compress/hist.c:29-164
 *
 * Everything is integer arithmetic; the output must equal the reference byte for byte
 * (tests/test_zstd_oracle.py checks it against oracle/_ref/libref.so, the reference compiled
 * from /root/reference, and against the committed golden frames).
 */
#include "oracle.h"
#include <stdlib.h>
#include <string.h>

typedef uint8_t u8;
typedef uint16_t u16;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int16_t s16;

static u32 hb32(u32 v) { return 31u - (u32)__builtin_clz(v); }
static u32 rd32(const u8* p) { u32 v; memcpy(&v, p, 4); return v; }
static u64 rd64(const u8* p) { u64 v; memcpy(&v, p, 8); return v; }
static void wr16(u8* p, u32 v) { p[0] = (u8)v; p[1] = (u8)(v >> 8); }
static void wr24(u8* p, u32 v) { p[0] = (u8)v; p[1] = (u8)(v >> 8); p[2] = (u8)(v >> 16); }
static void wr32(u8* p, u32 v) { wr16(p, v); wr16(p + 2, v >> 16); }

/* ------------------------------------------------------------------ format tables (RFC 8878) */
static const u8 LLB[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3,
                           4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const u8 MLB[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                           0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const s16 LL_DEF[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                               2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const s16 ML_DEF[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                               1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const s16 OF_DEF[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

/* literal-length / match-length codes (zstd_compress_internal.h:469-498) */
static u32 ll_code(u32 ll) {
    if (ll < 16) return ll;
    if (ll < 64) {   /* 16..63: pairs 16,17 -> 16 ... then 4-, 8-, 16-wide groups */
        static const u8 t[48] = {16, 16, 17, 17, 18, 18, 19, 19, 20, 20, 20, 20, 21, 21, 21, 21,
                                 22, 22, 22, 22, 22, 22, 22, 22, 23, 23, 23, 23, 23, 23, 23, 23,
                                 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24, 24};
        return t[ll - 16];
    }
    return hb32(ll) + 19;
}
static u32 ml_code(u32 mlBase) {
    static const u8 t[96] = {32, 32, 33, 33, 34, 34, 35, 35, 36, 36, 36, 36, 37, 37, 37, 37,
                             38, 38, 38, 38, 38, 38, 38, 38, 39, 39, 39, 39, 39, 39, 39, 39,
                             40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40, 40,
                             41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41, 41,
                             42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42,
                             42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42, 42};
    if (mlBase < 32) return mlBase;
    if (mlBase < 128) return t[mlBase - 32];
    return hb32(mlBase) + 36;
}

/* ------------------------------------------------------------------ parameters */
typedef struct { u32 wlog, hlog, mls, tlen; int fast; } zparams;

/* (W, H, minMatch, targetLength, strategy==fast) of clevels.h rows 0..2 per tableID */
static const u8 ROWS[4][3][5] = {
    {{19, 13, 6, 1, 1}, {19, 14, 7, 0, 1}, {20, 16, 6, 0, 1}},
    {{18, 13, 5, 1, 1}, {18, 14, 6, 0, 1}, {18, 16, 5, 0, 0}},
    {{17, 12, 5, 1, 1}, {17, 13, 6, 0, 1}, {17, 15, 5, 0, 1}},
    {{14, 13, 5, 1, 1}, {14, 15, 5, 0, 1}, {14, 15, 4, 0, 1}},
};

static int get_params(int level, size_t n, zparams* p) {
    const int unknown = (n == 0);   /* ZSTD_getParams: srcSizeHint 0 means unknown */
    const u32 tid = unknown ? 0 : (u32)(n <= 256 * 1024) + (n <= 128 * 1024) + (n <= 16 * 1024);
    int row = level < 0 ? 0 : level;
    if (row > 2) return -1;                                 /* only the fast-strategy rows */
    if (level == 0) return -1;                              /* (level 0 = default = 3: dfast) */
    const u8* r = ROWS[tid][row];
    if (!r[4]) return -1;
    p->wlog = r[0]; p->hlog = r[1]; p->mls = r[2]; p->tlen = r[3]; p->fast = 1;
    if (level < 0) p->tlen = (u32)(-(level < -131072 ? -131072 : level));
    if (!unknown && n < (1ull << 30)) {                     /* ZSTD_adjustCParams_internal */
        const u32 srcLog = n < 64 ? 6 : hb32((u32)(n - 1)) + 1;
        if (p->wlog > srcLog) p->wlog = srcLog;
    }
    if (!unknown && p->hlog > p->wlog + 1) p->hlog = p->wlog + 1;
    if (p->wlog < 10) p->wlog = 10;
    return 0;
}

/* ------------------------------------------------------------------ bit writer (LSB first) */
typedef struct { u8* out; size_t pos; u64 acc; u32 nb; } bitw;
static void bw_init(bitw* b, u8* out) { b->out = out; b->pos = 0; b->acc = 0; b->nb = 0; }
static void bw_add(bitw* b, u64 v, u32 n) {
    if (!n) return;
    v &= (n == 64) ? ~0ull : ((1ull << n) - 1);
    b->acc |= v << b->nb;
    b->nb += n;
    while (b->nb >= 8) { b->out[b->pos++] = (u8)b->acc; b->acc >>= 8; b->nb -= 8; }
}
/* end mark + padding: the stream size in bytes (BIT_closeCStream / HUF_closeCStream) */
static size_t bw_close(bitw* b) {
    bw_add(b, 1, 1);
    if (b->nb) { b->out[b->pos++] = (u8)b->acc; b->acc = 0; b->nb = 0; }
    return b->pos;
}

/* ------------------------------------------------------------------ histograms (hist.c) */
/* counts over [0..255]; *maxs = highest present symbol; returns the largest count */
static u32 histo(u32* cnt, u32 alphabet, u32* maxs, const u8* s, size_t n) {
    memset(cnt, 0, alphabet * sizeof(u32));
    if (!n) { *maxs = 0; return 0; }
    for (size_t i = 0; i < n; i++) cnt[s[i]]++;
    u32 m = alphabet - 1;
    while (!cnt[m]) m--;
    *maxs = m;
    u32 big = 0;
    for (u32 i = 0; i <= m; i++) if (cnt[i] > big) big = cnt[i];
    return big;
}

/* ------------------------------------------------------------------ FSE (fse_compress.c) */
typedef struct {
    u32 tlog;
    u16 st[1 << 12];        /* next-state table (tableSize entries) */
    int32_t dfs[256];       /* deltaFindState */
    u32 dnb[256];           /* deltaNbBits */
} fse_ct;

static u32 fse_min_log(size_t n, u32 maxs) {
    u32 a = hb32((u32)n) + 1, b = hb32(maxs) + 2;
    return a < b ? a : b;
}
/* FSE_optimalTableLog_internal (fse_compress.c:365-377) */
static u32 fse_opt_log(u32 maxLog, size_t n, u32 maxs, u32 minus) {
    u32 srcBits = hb32((u32)(n - 1)) - minus;
    u32 tl = maxLog ? maxLog : 11;
    u32 mb = fse_min_log(n, maxs);
    if (srcBits < tl) tl = srcBits;
    if (mb > tl) tl = mb;
    if (tl < 5) tl = 5;
    if (tl > 12) tl = 12;
    return tl;
}

/* secondary normalisation (FSE_normalizeM2, fse_compress.c:387-471) */
static int fse_norm_m2(s16* norm, u32 tl, const u32* cnt, size_t total, u32 maxs, s16 low) {
    const s16 NA = -2;
    u32 distributed = 0;
    u32 lowThreshold = (u32)(total >> tl);
    u32 lowOne = (u32)((total * 3) >> (tl + 1));
    for (u32 s = 0; s <= maxs; s++) {
        if (cnt[s] == 0) { norm[s] = 0; continue; }
        if (cnt[s] <= lowThreshold) { norm[s] = low; distributed++; total -= cnt[s]; continue; }
        if (cnt[s] <= lowOne) { norm[s] = 1; distributed++; total -= cnt[s]; continue; }
        norm[s] = NA;
    }
    u32 toDist = (1u << tl) - distributed;
    if (toDist == 0) return 0;
    if ((total / toDist) > lowOne) {
        lowOne = (u32)((total * 3) / (toDist * 2));
        for (u32 s = 0; s <= maxs; s++)
            if (norm[s] == NA && cnt[s] <= lowOne) { norm[s] = 1; distributed++; total -= cnt[s]; }
        toDist = (1u << tl) - distributed;
    }
    if (distributed == maxs + 1) {
        u32 mv = 0, mc = 0;
        for (u32 s = 0; s <= maxs; s++) if (cnt[s] > mc) { mv = s; mc = cnt[s]; }
        norm[mv] += (s16)toDist;
        return 0;
    }
    if (total == 0) {
        for (u32 s = 0; toDist > 0; s = (s + 1) % (maxs + 1))
            if (norm[s] > 0) { toDist--; norm[s]++; }
        return 0;
    }
    {
        const u64 vlog = 62 - tl;
        const u64 mid = (1ull << (vlog - 1)) - 1;
        const u64 rstep = (((1ull << vlog) * toDist) + mid) / (u32)total;
        u64 acc = mid;
        for (u32 s = 0; s <= maxs; s++) {
            if (norm[s] == NA) {
                const u64 end = acc + cnt[s] * rstep;
                const u32 w = (u32)(end >> vlog) - (u32)(acc >> vlog);
                if (w < 1) return -1;
                norm[s] = (s16)w;
                acc = end;
            }
        }
    }
    return 0;
}

/* FSE_normalizeCount (fse_compress.c:473-533); returns 0 on success */
static int fse_normalize(s16* norm, u32 tl, const u32* cnt, size_t total, u32 maxs, int useLow) {
    static const u32 rtb[8] = {0, 473195, 504333, 520860, 550000, 700000, 750000, 830000};
    if (tl < fse_min_log(total, maxs)) return -1;
    const s16 low = useLow ? -1 : 1;
    const u64 scale = 62 - tl;
    const u64 step = (1ull << 62) / (u32)total;
    const u64 vstep = 1ull << (scale - 20);
    int still = 1 << tl;
    u32 largest = 0;
    s16 largestP = 0;
    const u32 lowThreshold = (u32)(total >> tl);
    for (u32 s = 0; s <= maxs; s++) {
        if (cnt[s] == total) return 0;       /* rle: not reached (callers check) */
        if (cnt[s] == 0) { norm[s] = 0; continue; }
        if (cnt[s] <= lowThreshold) { norm[s] = low; still--; continue; }
        s16 p = (s16)((cnt[s] * step) >> scale);
        if (p < 8) {
            const u64 rest = vstep * rtb[p];
            p += (s16)((cnt[s] * step) - ((u64)p << scale) > rest);
        }
        if (p > largestP) { largestP = p; largest = s; }
        norm[s] = p;
        still -= p;
    }
    if (-still >= (norm[largest] >> 1)) return fse_norm_m2(norm, tl, cnt, total, maxs, low);
    norm[largest] += (s16)still;
    return 0;
}

/* FSE_writeNCount (fse_compress.c:232-325); returns bytes written */
static size_t fse_write_ncount(u8* out, const s16* norm, u32 maxs, u32 tl) {
    u8* o = out;
    const int tsize = 1 << tl;
    u32 bits = 0;
    int nb = 0;
    bits += (tl - 5) << nb;
    nb += 4;
    int remaining = tsize + 1, threshold = tsize, nbBits = (int)tl + 1;
    u32 sym = 0;
    const u32 alpha = maxs + 1;
    int prev0 = 0;
    while (sym < alpha && remaining > 1) {
        if (prev0) {
            u32 start = sym;
            while (sym < alpha && !norm[sym]) sym++;
            if (sym == alpha) break;
            while (sym >= start + 24) {
                start += 24;
                bits += 0xFFFFu << nb;
                o[0] = (u8)bits; o[1] = (u8)(bits >> 8); o += 2;
                bits >>= 16;
            }
            while (sym >= start + 3) { start += 3; bits += 3u << nb; nb += 2; }
            bits += (sym - start) << nb;
            nb += 2;
            if (nb > 16) { o[0] = (u8)bits; o[1] = (u8)(bits >> 8); o += 2; bits >>= 16; nb -= 16; }
        }
        {
            int c = norm[sym++];
            const int mx = (2 * threshold - 1) - remaining;
            remaining -= c < 0 ? -c : c;
            c++;
            if (c >= threshold) c += mx;
            bits += (u32)c << nb;
            nb += nbBits;
            nb -= (c < mx);
            prev0 = (c == 1);
            while (remaining < threshold) { nbBits--; threshold >>= 1; }
        }
        if (nb > 16) { o[0] = (u8)bits; o[1] = (u8)(bits >> 8); o += 2; bits >>= 16; nb -= 16; }
    }
    o[0] = (u8)bits; o[1] = (u8)(bits >> 8);
    o += (nb + 7) / 8;
    return (size_t)(o - out);
}

/* FSE_buildCTable_wksp (fse_compress.c:67-199) */
static void fse_build(fse_ct* ct, const s16* norm, u32 maxs, u32 tl) {
    const u32 tsize = 1u << tl, mask = tsize - 1, step = (tsize >> 1) + (tsize >> 3) + 3;
    u32 cumul[257];
    u8 sym_at[1 << 12];
    u32 high = tsize - 1;
    ct->tlog = tl;
    cumul[0] = 0;
    for (u32 u = 1; u <= maxs + 1; u++) {
        if (norm[u - 1] == -1) { cumul[u] = cumul[u - 1] + 1; sym_at[high--] = (u8)(u - 1); }
        else cumul[u] = cumul[u - 1] + (u32)norm[u - 1];
    }
    /* spread: the k-th placed occurrence lands at k*step, skipping the low-probability area */
    u32 pos = 0;
    for (u32 s = 0; s <= maxs; s++)
        for (int k = 0; k < norm[s]; k++) {
            sym_at[pos] = (u8)s;
            pos = (pos + step) & mask;
            while (pos > high) pos = (pos + step) & mask;
        }
    for (u32 u = 0; u < tsize; u++) ct->st[cumul[sym_at[u]]++] = (u16)(tsize + u);
    u32 total = 0;
    for (u32 s = 0; s <= maxs; s++) {
        const int c = norm[s];
        if (c == 0) { ct->dnb[s] = ((tl + 1) << 16) - (1u << tl); ct->dfs[s] = 0; }
        else if (c == -1 || c == 1) { ct->dnb[s] = (tl << 16) - (1u << tl); ct->dfs[s] = (int32_t)total - 1; total++; }
        else {
            const u32 mbo = tl - hb32((u32)c - 1);
            const u32 msp = (u32)c << mbo;
            ct->dnb[s] = (mbo << 16) - msp;
            ct->dfs[s] = (int32_t)total - c;
            total += (u32)c;
        }
    }
}

/* FSE_buildCTable_rle: table log 0, a single state */
static void fse_build_rle(fse_ct* ct, u32 sym) {
    ct->tlog = 0;
    ct->st[0] = 0;
    ct->dnb[sym] = 0;
    ct->dfs[sym] = 0;
}

static u32 fse_init_state(const fse_ct* ct, u32 sym) {          /* FSE_initCState2 */
    const u32 nbo = (ct->dnb[sym] + (1u << 15)) >> 16;
    const u32 v = (nbo << 16) - ct->dnb[sym];
    return ct->st[(int32_t)(v >> nbo) + ct->dfs[sym]];
}
static void fse_encode(bitw* b, const fse_ct* ct, u32* state, u32 sym) {   /* FSE_encodeSymbol */
    const u32 nbo = (*state + ct->dnb[sym]) >> 16;
    bw_add(b, *state, nbo);
    *state = ct->st[(int32_t)(*state >> nbo) + ct->dfs[sym]];
}

/* ------------------------------------------------------------------ Huffman (huf_compress.c) */
typedef struct { u32 count; u16 parent; u8 byte; u8 nbBits; } hnode;
typedef struct { u8 nb[256]; u16 val[256]; u32 tlog; } huf_ct;

/* sort symbols by decreasing count: buckets per distinct small count, log2 buckets from 165 on,
 * each log2 bucket quick-sorted (HUF_sort / HUF_simpleQuickSort, huf_compress.c:460-595).  The cutoff
 * RANK_POSITION_DISTINCT_COUNT_CUTOFF (huf_compress.c:455) is 158 + BIT_highbit32(158) = 165, not the 166
 * its comment states.  HUF_sort stores a symbol at region HUF_getIndex(count) + 1 (huf_compress.c:577), so the
 * reference's sort loop starts at region 165, which holds the count-164 ties (sorting them changes nothing),
 * and counts 165..255 are its region 166.  Buckets here are the reference's regions minus one: bucket 165
 * holds counts 165..255, and the sorted buckets start there */
static u32 huf_bucket(u32 c) { return c < 165 ? c : hb32(c) + 158; }
static void hn_swap(hnode* a, hnode* b) { hnode t = *a; *a = *b; *b = t; }
static void huf_isort(hnode* a, int lo, int hi) {
    const int size = hi - lo + 1;
    a += lo;
    for (int i = 1; i < size; i++) {
        const hnode key = a[i];
        int j = i - 1;
        while (j >= 0 && a[j].count < key.count) { a[j + 1] = a[j]; j--; }
        a[j + 1] = key;
    }
}
static int huf_partition(hnode* a, int lo, int hi) {
    const u32 pivot = a[hi].count;
    int i = lo - 1;
    for (int j = lo; j < hi; j++)
        if (a[j].count > pivot) { i++; hn_swap(&a[i], &a[j]); }
    hn_swap(&a[i + 1], &a[hi]);
    return i + 1;
}
static void huf_qsort(hnode* a, int lo, int hi) {
    if (hi - lo < 8) { huf_isort(a, lo, hi); return; }
    while (lo < hi) {
        const int p = huf_partition(a, lo, hi);
        if (p - lo < hi - p) { huf_qsort(a, lo, p - 1); lo = p + 1; }
        else { huf_qsort(a, p + 1, hi); hi = p - 1; }
    }
}
static void huf_sort(hnode* node, const u32* cnt, u32 maxs) {
    u16 base[192], cur[192];
    memset(base, 0, sizeof(base));
    for (u32 s = 0; s <= maxs; s++) base[huf_bucket(cnt[s])]++;
    for (int b = 191; b > 0; b--) { base[b - 1] += base[b]; cur[b - 1] = base[b - 1]; }
    cur[191] = base[191];
    for (u32 s = 0; s <= maxs; s++) {
        const u32 r = huf_bucket(cnt[s]) + 1;
        const u32 p = cur[r]++;
        node[p].count = cnt[s];
        node[p].byte = (u8)s;
    }
    for (u32 b = 165; b < 191; b++) {
        const u32 sz = (u32)cur[b] - base[b];
        if (sz > 1) huf_qsort(node + base[b], 0, (int)sz - 1);
    }
}

/* HUF_setMaxHeight (huf_compress.c:308-428) */
static u32 huf_limit(hnode* node, u32 last, u32 maxNb) {
    const u32 largest = node[last].nbBits;
    if (largest <= maxNb) return largest;
    int cost = 0;
    const u32 baseCost = 1u << (largest - maxNb);
    int n = (int)last;
    while (node[n].nbBits > maxNb) {
        cost += (int)(baseCost - (1u << (largest - node[n].nbBits)));
        node[n].nbBits = (u8)maxNb;
        n--;
    }
    while (node[n].nbBits == maxNb) n--;
    cost >>= (largest - maxNb);
    {
        const u32 NONE = 0xF0F0F0F0u;
        u32 rankLast[14];
        for (int i = 0; i < 14; i++) rankLast[i] = NONE;
        u32 curNb = maxNb;
        for (int p = n; p >= 0; p--) {
            if (node[p].nbBits >= curNb) continue;
            curNb = node[p].nbBits;
            rankLast[maxNb - curNb] = (u32)p;
        }
        while (cost > 0) {
            u32 dec = hb32((u32)cost) + 1;
            for (; dec > 1; dec--) {
                const u32 hi = rankLast[dec], lo = rankLast[dec - 1];
                if (hi == NONE) continue;
                if (lo == NONE) break;
                if (node[hi].count <= 2 * node[lo].count) break;
            }
            while (dec <= 12 && rankLast[dec] == NONE) dec++;
            cost -= 1 << (dec - 1);
            node[rankLast[dec]].nbBits++;
            if (rankLast[dec - 1] == NONE) rankLast[dec - 1] = rankLast[dec];
            if (rankLast[dec] == 0) rankLast[dec] = NONE;
            else {
                rankLast[dec]--;
                if (node[rankLast[dec]].nbBits != maxNb - dec) rankLast[dec] = NONE;
            }
        }
        while (cost < 0) {
            if (rankLast[1] == NONE) {
                while (node[n].nbBits == maxNb) n--;
                node[n + 1].nbBits--;
                rankLast[1] = (u32)(n + 1);
                cost++;
                continue;
            }
            node[rankLast[1] + 1].nbBits--;
            rankLast[1]++;
            cost++;
        }
    }
    return maxNb;
}

/* HUF_buildCTable_wksp (huf_compress.c:610-708): returns the table log actually used */
static u32 huf_build(huf_ct* ct, const u32* cnt, u32 maxs, u32 maxNb) {
    hnode all[2 * 256 + 2];
    memset(all, 0, sizeof(all));
    hnode* node = all + 1;
    huf_sort(node, cnt, maxs);
    /* tree (HUF_buildTree): leaves node[0..nonNull], internal nodes from 256 upward */
    int nonNull = (int)maxs;
    while (node[nonNull].count == 0) nonNull--;
    int lowS = nonNull, nodeNb = 256;
    const int root = nodeNb + lowS - 1;
    int lowN = nodeNb;
    node[nodeNb].count = node[lowS].count + node[lowS - 1].count;
    node[lowS].parent = node[lowS - 1].parent = (u16)nodeNb;
    nodeNb++;
    lowS -= 2;
    for (int i = nodeNb; i <= root; i++) node[i].count = 1u << 30;
    all[0].count = 1u << 31;
    while (nodeNb <= root) {
        const int a = (node[lowS].count < node[lowN].count) ? lowS-- : lowN++;
        const int b = (node[lowS].count < node[lowN].count) ? lowS-- : lowN++;
        node[nodeNb].count = node[a].count + node[b].count;
        node[a].parent = node[b].parent = (u16)nodeNb;
        nodeNb++;
    }
    node[root].nbBits = 0;
    for (int i = root - 1; i >= 256; i--) node[i].nbBits = node[node[i].parent].nbBits + 1;
    for (int i = 0; i <= nonNull; i++) node[i].nbBits = node[node[i].parent].nbBits + 1;
    maxNb = huf_limit(node, (u32)nonNull, maxNb);
    /* canonical codes (HUF_buildCTableFromTree) */
    u16 nbPer[13] = {0}, valPer[13] = {0};
    for (int i = 0; i <= nonNull; i++) nbPer[node[i].nbBits]++;
    u16 mn = 0;
    for (int b = (int)maxNb; b > 0; b--) { valPer[b] = mn; mn += nbPer[b]; mn >>= 1; }
    memset(ct->nb, 0, sizeof(ct->nb));
    memset(ct->val, 0, sizeof(ct->val));
    for (u32 i = 0; i <= maxs; i++) ct->nb[node[i].byte] = node[i].nbBits;
    for (u32 s = 0; s <= maxs; s++) if (ct->nb[s]) ct->val[s] = valPer[ct->nb[s]]++; else valPer[0]++;
    ct->tlog = maxNb;
    return maxNb;
}

static size_t huf_estimate(const huf_ct* ct, const u32* cnt, u32 maxs) {
    size_t bits = 0;
    for (u32 s = 0; s <= maxs; s++) bits += (size_t)ct->nb[s] * cnt[s];
    return bits >> 3;
}
static int huf_valid(const huf_ct* ct, const u32* cnt, u32 maxs) {
    for (u32 s = 0; s <= maxs; s++) if (cnt[s] && !ct->nb[s]) return 0;
    return 1;
}

/* FSE compression of the Huffman weights (HUF_compressWeights, huf_compress.c:92-129 +
 * FSE_compress_usingCTable_generic, fse_compress.c:593-650); 0 = not compressible, 1 = rle */
static size_t huf_compress_weights(u8* out, const u8* w, u32 wn) {
    if (wn <= 1) return 0;
    u32 cnt[13], maxs;
    u32 big = histo(cnt, 13, &maxs, w, wn);
    if (big == wn) return 1;
    if (big == 1) return 0;
    const u32 tl = fse_opt_log(6, wn, maxs, 2);
    s16 norm[13];
    if (fse_normalize(norm, tl, cnt, wn, maxs, 0)) return 0;
    size_t h = fse_write_ncount(out, norm, maxs, tl);
    fse_ct ct;
    fse_build(&ct, norm, maxs, tl);
    if (wn <= 2) return 0;
    bitw b;
    bw_init(&b, out + h);
    u32 s1, s2;
    int i = (int)wn;
    if (wn & 1) {
        s1 = fse_init_state(&ct, w[--i]);
        s2 = fse_init_state(&ct, w[--i]);
        fse_encode(&b, &ct, &s1, w[--i]);
    } else {
        s2 = fse_init_state(&ct, w[--i]);
        s1 = fse_init_state(&ct, w[--i]);
    }
    while (i > 0) {    /* alternate states, last symbol first */
        fse_encode(&b, &ct, &s2, w[--i]);
        fse_encode(&b, &ct, &s1, w[--i]);
    }
    bw_add(&b, s2, ct.tlog);
    bw_add(&b, s1, ct.tlog);
    return h + bw_close(&b);
}

/* HUF_writeCTable_wksp (huf_compress.c:172-208); < 0 = error */
static long huf_write_table(u8* out, const huf_ct* ct, u32 maxs, u32 tlog) {
    u8 w[256];
    for (u32 s = 0; s < maxs; s++) w[s] = ct->nb[s] ? (u8)(tlog + 1 - ct->nb[s]) : 0;
    size_t h = huf_compress_weights(out + 1, w, maxs);
    if (h > 1 && h < maxs / 2) { out[0] = (u8)h; return (long)h + 1; }
    if (maxs > 128) return -1;
    out[0] = (u8)(128 + maxs - 1);
    w[maxs] = 0;
    for (u32 s = 0; s < maxs; s += 2) out[s / 2 + 1] = (u8)((w[s] << 4) + w[s + 1]);
    return (long)((maxs + 1) / 2 + 1);
}

/* one Huffman stream: symbols last to first, then the end mark (HUF_compress1X_usingCTable) */
static size_t huf_stream(u8* out, const u8* s, size_t n, const huf_ct* ct) {
    bitw b;
    bw_init(&b, out);
    for (size_t i = n; i-- > 0;) bw_add(&b, ct->val[s[i]], ct->nb[s[i]]);
    return bw_close(&b);
}
static size_t huf_streams(u8* out, const u8* s, size_t n, const huf_ct* ct, int four) {
    if (!four) return huf_stream(out, s, n, ct);
    if (n < 12) return 0;
    const size_t seg = (n + 3) / 4;
    size_t o = 6;
    for (int k = 0; k < 4; k++) {
        const size_t len = k < 3 ? seg : n - 3 * seg;
        const size_t c = huf_stream(out + o, s + k * seg, len, ct);
        if (c == 0 || c > 65535) return 0;
        if (k < 3) wr16(out + 2 * k, (u32)c);
        o += c;
    }
    return o;
}

typedef struct { huf_ct ct; int repeat; /* 0 none, 1 check */ } huf_state;

/* HUF_compress_internal (huf_compress.c:1177-1282) for the fast strategy.  Returns the size
 * of header + streams, 0 = not compressible, 1 = rle; *reused = previous table kept. */
static long huf_compress(u8* out, const u8* src, size_t n, int four, huf_state* prev, huf_state* next,
                         int* reused, int suspect) {
    *reused = 0;
    if (!n) return 0;
    u32 cnt[256], maxs = 255;
    if (suspect && n >= 4096 * 10) {
        u32 m1, m2;
        size_t big = histo(cnt, 256, &m1, src, 4096);
        big += histo(cnt, 256, &m2, src + n - 4096, 4096);
        if (big <= ((2 * 4096) >> 7) + 4) return 0;
    }
    const u32 big = histo(cnt, 256, &maxs, src, n);
    if (big == n) { out[0] = src[0]; return 1; }
    if (big <= (n >> 7) + 4) return 0;
    int repeat = prev->repeat;
    if (repeat && !huf_valid(&prev->ct, cnt, maxs)) repeat = 0;
    const int preferRepeat = n <= 1024;
    if (preferRepeat && repeat) {
        *reused = 1;
        size_t c = huf_streams(out, src, n, &prev->ct, four);
        return (c == 0 || c >= n - 1) ? 0 : (long)c;
    }
    huf_ct fresh;
    const u32 tl = huf_build(&fresh, cnt, maxs, fse_opt_log(11, n, maxs, 1));
    u8 hdr[256];
    const long h = huf_write_table(hdr, &fresh, maxs, tl);
    if (h < 0) return -1;
    if (repeat) {
        const size_t oldS = huf_estimate(&prev->ct, cnt, maxs), newS = huf_estimate(&fresh, cnt, maxs);
        if (oldS <= (size_t)h + newS || (size_t)h + 12 >= n) {
            *reused = 1;
            size_t c = huf_streams(out, src, n, &prev->ct, four);
            return (c == 0 || c >= n - 1) ? 0 : (long)c;
        }
    }
    if ((size_t)h + 12 >= n) return 0;
    memcpy(out, hdr, (size_t)h);
    next->ct = fresh;
    size_t c = huf_streams(out + h, src, n, &fresh, four);
    if (c == 0 || (size_t)h + c >= n - 1) return 0;
    return h + (long)c;
}

/* ZSTD_compressLiterals (zstd_compress_literals.c:70-159) */
static size_t lit_raw(u8* out, const u8* src, size_t n) {
    const u32 fl = 1 + (n > 31) + (n > 4095);
    if (fl == 1) out[0] = (u8)(n << 3);
    else if (fl == 2) wr16(out, (u32)(1 << 2) + (u32)(n << 4));
    else wr24(out, (u32)(3 << 2) + (u32)(n << 4));
    memcpy(out + fl, src, n);
    return n + fl;
}
static size_t lit_rle(u8* out, u8 b, size_t n) {
    const u32 fl = 1 + (n > 31) + (n > 4095);
    if (fl == 1) out[0] = (u8)(1 + (n << 3));
    else if (fl == 2) wr16(out, 1 + (u32)(1 << 2) + (u32)(n << 4));
    else wr24(out, 1 + (u32)(3 << 2) + (u32)(n << 4));
    out[fl] = b;
    return fl + 1;
}
static size_t compress_literals(u8* out, const u8* src, size_t n, huf_state* prev, huf_state* next, int disable,
                                int suspect) {
    *next = *prev;
    if (disable || n <= 63) return lit_raw(out, src, n);
    const size_t lh = 3 + (n >= 1024) + (n >= 16 * 1024);
    const int single = n < 256;
    int reused = 0;
    huf_state tmp = *prev;
    const long c = huf_compress(out + lh, src, n, !single, prev, &tmp, &reused, suspect);
    const size_t minGain = (n >> 6) + 2;
    if (c <= 0 || (size_t)c >= n - minGain) { *next = *prev; return lit_raw(out, src, n); }
    if (c == 1) { *next = *prev; return lit_rle(out, src[0], n); }
    u32 htype = 3;                         /* set_repeat */
    if (!reused) { htype = 2; next->ct = tmp.ct; next->repeat = 1; }
    if (lh == 3) wr24(out, htype + ((u32)(!single) << 2) + ((u32)n << 4) + ((u32)c << 14));
    else if (lh == 4) wr32(out, htype + (2u << 2) + ((u32)n << 4) + ((u32)c << 18));
    else { wr32(out, htype + (3u << 2) + ((u32)n << 4) + ((u32)c << 22)); out[4] = (u8)(c >> 10); }
    return lh + (size_t)c;
}

/* ------------------------------------------------------------------ sequences */
typedef struct { u32 ll, off, ml; } zseq;   /* literal length, offBase (1 = repcode 1), match length */

/* ZSTD_selectEncodingType for strategies below lazy (zstd_compress_sequences.c:157-235);
 * the fast strategy never sees a valid repeat table, so set_repeat does not arise.
 * 0 basic, 1 rle, 2 compressed */
static int select_type(u32 mostFrequent, size_t nbSeq, u32 defLog, int defAllowed) {
    if (mostFrequent == nbSeq) return (defAllowed && nbSeq <= 2) ? 0 : 1;
    if (defAllowed) {
        const size_t dynMin = ((size_t)(1u << defLog) * 9) >> 3;   /* mult = 10 - ZSTD_fast */
        if (nbSeq < dynMin || mostFrequent < (nbSeq >> (defLog - 1))) return 0;
    }
    return 2;
}

/* the sequences section after the nbSeq header; returns its size or 0 for "emit raw" */
static size_t encode_sequences(u8* out, const zseq* seq, size_t nbSeq) {
    u8* op = out;
    u8* llc = (u8*)malloc(nbSeq), *ofc = (u8*)malloc(nbSeq), *mlc = (u8*)malloc(nbSeq);
    for (size_t i = 0; i < nbSeq; i++) {
        llc[i] = (u8)ll_code(seq[i].ll);
        ofc[i] = (u8)hb32(seq[i].off);
        mlc[i] = (u8)ml_code(seq[i].ml - 3);
    }
    fse_ct ct[3];   /* (on the stack: the _mt chunk loops call this from several threads) */
    const u8* codes[3] = {llc, ofc, mlc};
    const u32 maxTab[3] = {35, 31, 52}, fseLog[3] = {9, 8, 9}, defLog[3] = {6, 5, 6}, defMax[3] = {35, 28, 52};
    const s16* defNorm[3] = {LL_DEF, OF_DEF, ML_DEF};
    u8* head = op++;
    u32 types[3];
    size_t lastCount = 0;
    for (int t = 0; t < 3; t++) {
        u32 cnt[64], maxs;
        const u32 big = histo(cnt, maxTab[t] + 1, &maxs, codes[t], nbSeq);
        const int defOk = t == 1 ? (maxs <= 28) : 1;
        const int ty = select_type(big, nbSeq, defLog[t], defOk);
        types[t] = (u32)ty;
        if (ty == 1) { fse_build_rle(&ct[t], maxs); *op++ = codes[t][0]; }
        else if (ty == 0) fse_build(&ct[t], defNorm[t], defMax[t], defLog[t]);
        else {
            size_t n1 = nbSeq;
            const u32 tl = fse_opt_log(fseLog[t], nbSeq, maxs, 2);
            if (cnt[codes[t][nbSeq - 1]] > 1) { cnt[codes[t][nbSeq - 1]]--; n1--; }
            s16 norm[64];
            fse_normalize(norm, tl, cnt, n1, maxs, n1 >= 2048);
            const size_t h = fse_write_ncount(op, norm, maxs, tl);
            fse_build(&ct[t], norm, maxs, tl);
            op += h;
            lastCount = h;
        }
    }
    *head = (u8)((types[0] << 6) + (types[1] << 4) + (types[2] << 2));
    /* ZSTD_encodeSequences_body (zstd_compress_sequences.c:290-382) */
    bitw b;
    bw_init(&b, op);
    const size_t L = nbSeq - 1;
    u32 sML = fse_init_state(&ct[2], mlc[L]);
    u32 sOF = fse_init_state(&ct[1], ofc[L]);
    u32 sLL = fse_init_state(&ct[0], llc[L]);
    bw_add(&b, seq[L].ll, LLB[llc[L]]);
    bw_add(&b, seq[L].ml - 3, MLB[mlc[L]]);
    bw_add(&b, seq[L].off, ofc[L]);
    for (size_t n = nbSeq - 1; n-- > 0;) {
        fse_encode(&b, &ct[1], &sOF, ofc[n]);
        fse_encode(&b, &ct[2], &sML, mlc[n]);
        fse_encode(&b, &ct[0], &sLL, llc[n]);
        bw_add(&b, seq[n].ll, LLB[llc[n]]);
        bw_add(&b, seq[n].ml - 3, MLB[mlc[n]]);
        bw_add(&b, seq[n].off, ofc[n]);
    }
    bw_add(&b, sML, ct[2].tlog);
    bw_add(&b, sOF, ct[1].tlog);
    bw_add(&b, sLL, ct[0].tlog);
    const size_t bs = bw_close(&b);
    free(llc); free(ofc); free(mlc);
    if (lastCount && lastCount + bs < 4) return 0;    /* zstd <= 1.3.4 decoder workaround */
    return (size_t)(op - out) + bs;
}

/* ------------------------------------------------------------------ match finder (zstd_fast.c) */
typedef struct {
    u32* table;
    u32 hlog, mls;
    const u8* base;          /* frame start: index 0 */
} mstate;

static u32 zhash(const u8* p, u32 hlog, u32 mls) {
    const u64 v = rd64(p);
    switch (mls) {
        case 5: return (u32)(((v << 24) * 889523592379ull) >> (64 - hlog));
        case 6: return (u32)(((v << 16) * 227718039650203ull) >> (64 - hlog));
        case 7: return (u32)(((v << 8) * 58295818150454627ull) >> (64 - hlog));
        default: return (u32)((u32)v * 2654435761u) >> (32 - hlog);
    }
}
static size_t zcount(const u8* a, const u8* b, const u8* end) {
    size_t n = 0;
    while (a + n < end && a[n] == b[n]) n++;
    return n;
}

/* One block [bs, be) of the frame (positions are byte offsets from the frame start; the
 * reference's table indices are these plus a constant, entries below the frame start are
 * invalid).  Table semantics per probed position q: read T[h(q)], then write T[h(q)] = q. */
static size_t fast_block(mstate* m, size_t bs, size_t be, u32 rep[2], u32 stepSize, size_t W, zseq* seq,
                         size_t* nseq, u8* lits, size_t* nlit) {
    const u8* src = m->base;
    const size_t ilimit = be >= 8 ? be - 8 : 0;
    u32* T = m->table;
    const u32 hl = m->hlog, ml = m->mls;
    /* table entries are stored +1 so that 0 means "never written" (below the prefix) */
#define TGET(q) (T[zhash(src + (q), hl, ml)])
#define TSET(q) (T[zhash(src + (q), hl, ml)] = (u32)(q) + 1)
    /* window (W = 2^windowLog): ZSTD_window_enforceMaxDist at the block start raises the lowest
     * valid position to bs - W (zstd_compress.c:3962), and ZSTD_getLowestPrefixIndex for the block
     * end gives the prefix start the match finder validates candidates against (zstd_fast.c:106) */
    const size_t dl = bs > W ? bs - W : 0;
    const size_t pstart = (be - dl > W) ? be - W : dl;
    size_t ip = bs + (bs == pstart);
    size_t anchor = bs;
    u32 r1 = rep[0], r2 = rep[1], saved = 0;
    {
        const size_t wlow = (ip - dl > W) ? ip - W : dl;
        const u32 maxRep = (u32)(ip - wlow);
        if (r2 > maxRep) { saved = r2; r2 = 0; }
        if (r1 > maxRep) { saved = r1; r1 = 0; }
    }
    size_t ns = 0, nl = 0;
    if (be - bs < 8) goto done;   /* (callers never pass such blocks) */
    for (;;) {
        /* _start: search from ip */
        size_t A = ip;
        u32 D = stepSize, step = stepSize;
        size_t nextStep = A + 128;
        if (A + stepSize + 1 >= ilimit) break;
        size_t mstart = 0, mpos = 0, ip1 = 0, cur0 = 0;
        int kind = 0;   /* 1 rep at A+D, 2 regular at A, 3 regular at A+1 */
        for (;;) {
            const u32 c0 = TGET(A);
            TSET(A);
            if (r1 > 0 && rd32(src + A + D) == rd32(src + A + D - r1)) { kind = 1; cur0 = A; ip1 = A + 1; break; }
            if (c0 > pstart && rd32(src + c0 - 1) == rd32(src + A)) { kind = 2; mpos = c0 - 1; cur0 = A; ip1 = A + 1; break; }
            const u32 c1 = TGET(A + 1);
            TSET(A + 1);
            if (c1 > pstart && rd32(src + c1 - 1) == rd32(src + A + 1)) { kind = 3; mpos = c1 - 1; cur0 = A + 1; ip1 = A + D; break; }
            const size_t An = A + D;
            const u32 Dn = step;
            if (An + step >= nextStep) { step++; nextStep += 128; }
            if (An + 1 + Dn >= ilimit) goto done;
            A = An;
            D = Dn;
        }
        size_t len;
        u32 offBase;
        if (kind == 1) {
            mstart = A + D;
            mpos = mstart - r1;
            const size_t back = src[mstart - 1] == src[mpos - 1];
            mstart -= back;
            mpos -= back;
            len = 4 + back;
            offBase = 1;
        } else {
            mstart = kind == 2 ? A : A + 1;
            r2 = r1;
            r1 = (u32)(mstart - mpos);
            offBase = r1 + 3;
            len = 4;
            while (mstart > anchor && mpos > pstart && src[mstart - 1] == src[mpos - 1]) { mstart--; mpos--; len++; }
        }
        len += zcount(src + mstart + len, src + mpos + len, src + be);
        seq[ns].ll = (u32)(mstart - anchor); seq[ns].off = offBase; seq[ns].ml = (u32)len; ns++;
        memcpy(lits + nl, src + anchor, mstart - anchor);
        nl += mstart - anchor;
        ip = mstart + len;
        anchor = ip;
        if (ip1 < ip) TSET(ip1);
        if (ip <= ilimit) {
            TSET(cur0 + 2);
            TSET(ip - 2);
            if (r2 > 0) {
                while (ip <= ilimit && rd32(src + ip) == rd32(src + ip - r2)) {
                    const size_t rl = 4 + zcount(src + ip + 4, src + ip + 4 - r2, src + be);
                    const u32 t = r2; r2 = r1; r1 = t;
                    TSET(ip);
                    seq[ns].ll = 0; seq[ns].off = 1; seq[ns].ml = (u32)rl; ns++;
                    ip += rl;
                    anchor = ip;
                }
            }
        }
    }
done:
    rep[0] = r1 ? r1 : saved;
    rep[1] = r2 ? r2 : saved;
    memcpy(lits + nl, src + anchor, be - anchor);   /* last literals */
    nl += be - anchor;
    *nseq = ns;
    *nlit = nl;
#undef TGET
#undef TSET
    return 0;
}

/* ------------------------------------------------------------------ frame */
static int is_rle(const u8* s, size_t n) {
    for (size_t i = 1; i < n; i++) if (s[i] != s[0]) return 0;
    return 1;
}

size_t oracle_zstd_bound(size_t n) {
    return n + (n >> 8) + (n < (128u << 10) ? ((128u << 10) - n) >> 11 : 0);
}

int64_t oracle_zstd_compress(const uint8_t* src, size_t n, uint8_t* dst, int level) {
    zparams P;
    if (get_params(level, n, &P)) return -1;
    u8* op = dst;
    /* frame header (ZSTD_writeFrameHeader): magic, descriptor, single-segment content size */
    wr32(op, 0xFD2FB528u);
    op += 4;
    {
        const u32 wsize = 1u << P.wlog;
        const int single = wsize >= n;
        const u32 fcs = (n >= 256) + (n >= 65536 + 256) + (n >= 0xFFFFFFFFull);
        *op++ = (u8)((single << 5) + (fcs << 6));
        if (!single) *op++ = (u8)((P.wlog - 10) << 3);
        if (fcs == 0) { if (single) *op++ = (u8)n; }
        else if (fcs == 1) { wr16(op, (u32)(n - 256)); op += 2; }
        else if (fcs == 2) { wr32(op, (u32)n); op += 4; }
        else { wr32(op, (u32)n); wr32(op + 4, (u32)((u64)n >> 32)); op += 8; }
    }
    if (n == 0) {   /* ZSTD_writeEpilogue: an empty last raw block */
        wr24(op, 1);
        return (int64_t)(op + 3 - dst);
    }
    size_t wsz = (size_t)1 << P.wlog;
    size_t bsize = 128u << 10;
    if (wsz < bsize) bsize = wsz;
    if (n < bsize) bsize = n;
    mstate m;
    m.hlog = P.hlog;
    m.mls = P.mls;
    m.base = src;
    m.table = (u32*)calloc((size_t)1 << P.hlog, sizeof(u32));
    const u32 stepSize = P.tlen > 1 ? P.tlen + 1 : 2;      /* hasStep = targetLength > 1 */
    const int litDisabled = P.tlen > 0;                     /* fast && targetLength > 0 */
    u32 rep[2] = {1, 4};                                    /* repStartValue */
    huf_state hprev;
    memset(&hprev, 0, sizeof(hprev));
    zseq* seq = (zseq*)malloc((bsize / 3 + 16) * sizeof(zseq));
    u8* lits = (u8*)malloc(bsize + 16);
    u8* body = (u8*)malloc(bsize * 2 + 1024);
    int first = 1;
    for (size_t bs = 0; bs < n; bs += bsize) {
        const size_t be = bs + bsize < n ? bs + bsize : n;
        const size_t len = be - bs;
        const int last = be == n;
        size_t csize = 0;
        u32 nrep[2] = {rep[0], rep[1]};
        huf_state hnext = hprev;
        if (len >= 7) {   /* MIN_CBLOCK_SIZE + ZSTD_blockHeaderSize + 1 */
            size_t ns = 0, nl = 0;
            fast_block(&m, bs, be, nrep, stepSize, wsz, seq, &ns, lits, &nl);
            const int suspect = ns == 0 || nl / ns >= 20;
            u8* o = body;
            o += compress_literals(o, lits, nl, &hprev, &hnext, litDisabled, suspect);
            if (ns < 128) *o++ = (u8)ns;
            else if (ns < 0x7F00) { o[0] = (u8)((ns >> 8) + 0x80); o[1] = (u8)ns; o += 2; }
            else { o[0] = 0xFF; wr16(o + 1, (u32)(ns - 0x7F00)); o += 3; }
            if (ns) {
                const size_t s = encode_sequences(o, seq, ns);
                csize = s ? (size_t)(o - body) + s : 0;
            } else {
                csize = (size_t)(o - body);
            }
            if (csize && csize >= len - ((len >> 6) + 2)) csize = 0;      /* ZSTD_minGain */
        }
        if (len >= 7 && !first && csize < 25 && is_rle(src + bs, len)) csize = 1;
        if (csize == 0) {
            wr24(op, (u32)last + (u32)(len << 3));
            memcpy(op + 3, src + bs, len);
            op += 3 + len;
        } else if (csize == 1) {
            wr24(op, (u32)last + (1u << 1) + (u32)(len << 3));
            op[3] = src[bs];
            op += 4;
        } else {
            wr24(op, (u32)last + (2u << 1) + (u32)(csize << 3));
            memcpy(op + 3, body, csize);
            op += 3 + csize;
            rep[0] = nrep[0]; rep[1] = nrep[1];      /* confirm repcodes + entropy tables */
            hprev = hnext;
        }
        first = 0;
    }
    free(m.table); free(seq); free(lits); free(body);
    return (int64_t)(op - dst);
}
