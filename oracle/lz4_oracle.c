/*
 * oracle/lz4_oracle.c -- plain-C restatement of the LZ4 1.9.3 block codec as lzbench
 * drives it.  TEST INFRASTRUCTURE ONLY (see oracle.h): the checker for the HIP path.
 *
 * Restated from the reference algorithm, not copied:
 *   hash4 / hash5 ........................ /root/reference/lz4/lz4.c:698-722
 *   table type choice (byU16 < 65547 B) .. lz4.c:633, :1284-1305
 *   greedy parser ........................ lz4.c:851-1240 (noDict, notLimited)
 *   LZ4_count semantics .................. lz4.c:603-626 (= min(common prefix, limit-p))
 *   safe decoder acceptance rules ........ lz4.c:1707-1729, :1929-2151, :2170-2176
 */
#include "oracle.h"
#include <string.h>

#define LZ4O_MINMATCH 4
#define LZ4O_MFLIMIT 12
#define LZ4O_LASTLITERALS 5
#define LZ4O_MINLENGTH 13      /* MFLIMIT + 1 : shorter inputs are all literals */
#define LZ4O_LIMIT64K 65547    /* 64 KiB + MFLIMIT - 1 */

static uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t rd64(const uint8_t* p) { uint64_t v; memcpy(&v, p, 8); return v; }

int oracle_lz4_bound(int n) { return n + n / 255 + 16; }

typedef struct {
    int small;          /* 1: byU16 table of 8192 u16, hash4 >> 19; 0: byU32 table of 4096 u32, hash5 */
    uint16_t t16[1 << 13];
    uint32_t t32[1 << 12];
    const uint8_t* s;
} lz4o_tab;

static uint32_t lz4o_hash(const lz4o_tab* t, int pos) {
    if (t->small) return (rd32(t->s + pos) * 2654435761u) >> 19;
    return (uint32_t)(((rd64(t->s + pos) << 24) * 889523592379ull) >> 52);
}
static uint32_t lz4o_get(const lz4o_tab* t, uint32_t h) { return t->small ? t->t16[h] : t->t32[h]; }
static void lz4o_put(lz4o_tab* t, uint32_t h, uint32_t pos) {
    if (t->small) t->t16[h] = (uint16_t)pos; else t->t32[h] = pos;
}

/* number of equal bytes at a and b, not letting a run past limit */
static int lz4o_common(const uint8_t* s, int a, int b, int limit) {
    int k = 0;
    while (a + k < limit && s[a + k] == s[b + k]) k++;
    return k;
}

static int lz4o_put_len(uint8_t* dst, int op, int len) {
    /* 255-run length continuation: floor(len/255) bytes of 255 then len%255 */
    while (len >= 255) { dst[op++] = 255; len -= 255; }
    dst[op++] = (uint8_t)len;
    return op;
}

int oracle_lz4_compress(const uint8_t* src, int n, uint8_t* dst, int acceleration) {
    static __thread lz4o_tab tab;           /* 48 KiB, keep it off the stack */
    if (acceleration < 1) acceleration = 1;
    if (acceleration > 65537) acceleration = 65537;
    if (n <= 0) { dst[0] = 0; return 1; }

    lz4o_tab* t = &tab;
    t->small = n < LZ4O_LIMIT64K;
    t->s = src;
    if (t->small) memset(t->t16, 0, sizeof t->t16); else memset(t->t32, 0, sizeof t->t32);

    const int mfl1 = n - LZ4O_MFLIMIT + 1;      /* mflimitPlusOne */
    const int mlimit = n - LZ4O_LASTLITERALS;   /* matchlimit */
    int ip = 0, anchor = 0, op = 0;
    uint32_t fh;

    if (n < LZ4O_MINLENGTH) goto last_literals;

    lz4o_put(t, lz4o_hash(t, 0), 0);
    ip = 1;
    fh = lz4o_hash(t, ip);

    for (;;) {
        int match, tok;
        /* probe loop: positions advance by step, step grows every 64 probes */
        {
            int fwd = ip, step = 1, nb = acceleration << 6;
            for (;;) {
                uint32_t h = fh;
                int cur = fwd;
                uint32_t cand = lz4o_get(t, h);
                ip = fwd;
                fwd += step;
                step = nb++ >> 6;
                if (fwd > mfl1) goto last_literals;
                fh = lz4o_hash(t, fwd);
                lz4o_put(t, h, (uint32_t)cur);
                if (!t->small && cand + 65535u < (uint32_t)cur) continue;   /* too far */
                if (rd32(src + cand) == rd32(src + ip)) { match = (int)cand; break; }
            }
        }
        /* extend backwards over equal bytes */
        while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) { ip--; match--; }

        {   /* token + literal run */
            int lit = ip - anchor;
            tok = op++;
            if (lit >= 15) { dst[tok] = 15 << 4; op = lz4o_put_len(dst, op, lit - 15); }
            else dst[tok] = (uint8_t)(lit << 4);
            memcpy(dst + op, src + anchor, (size_t)lit);
            op += lit;
        }

    next_match:
        {
            int off = ip - match;
            dst[op++] = (uint8_t)(off & 0xff);
            dst[op++] = (uint8_t)(off >> 8);
            int ml = lz4o_common(src, ip + LZ4O_MINMATCH, match + LZ4O_MINMATCH, mlimit);
            ip += ml + LZ4O_MINMATCH;
            if (ml >= 15) { dst[tok] = (uint8_t)(dst[tok] + 15); op = lz4o_put_len(dst, op, ml - 15); }
            else dst[tok] = (uint8_t)(dst[tok] + ml);
        }
        anchor = ip;
        if (ip >= mfl1) break;

        lz4o_put(t, lz4o_hash(t, ip - 2), (uint32_t)(ip - 2));
        {   /* immediate re-test at the match end (no catch-up on this path) */
            uint32_t h = lz4o_hash(t, ip);
            uint32_t cand = lz4o_get(t, h);
            lz4o_put(t, h, (uint32_t)ip);
            if ((t->small || cand + 65535u >= (uint32_t)ip) && rd32(src + cand) == rd32(src + ip)) {
                match = (int)cand;
                tok = op++;
                dst[tok] = 0;
                goto next_match;
            }
        }
        ip++;
        fh = lz4o_hash(t, ip);
    }

last_literals:
    {
        int run = n - anchor;
        if (run >= 15) { dst[op++] = 15 << 4; op = lz4o_put_len(dst, op, run - 15); }
        else dst[op++] = (uint8_t)(run << 4);
        memcpy(dst + op, src + anchor, (size_t)run);
        op += run;
    }
    return op;
}

/* ---------------------------------------------------------------- decoder */

int oracle_lz4_decompress_safe(const uint8_t* src, int csize, uint8_t* dst, int cap) {
    return oracle_lz4_decompress_prefix(src, csize, dst, cap, 0);
}

/* the same with `prefix` bytes of earlier output before dst that matches may reach into
 * (LZ4_decompress_safe_usingDict in prefix mode, lz4.c:2404-2416; the offset check of
 * LZ4_decompress_generic then fails only below dst - prefix, :1915-1917) */
int oracle_lz4_decompress_prefix(const uint8_t* src, int csize, uint8_t* dst, int cap, int64_t prefix) {
    int64_t ip = 0, op = 0;
    const int64_t iend = csize, oend = cap;
    if (cap == 0) return (csize == 1 && src[0] == 0) ? 0 : -1;
    if (csize <= 0) return -1;
    for (;;) {
        if (ip >= iend) return (int)(-ip - 1);
        unsigned tok = src[ip++];
        int64_t lit = tok >> 4;
        if (lit == 15) {
            /* literal-length continuation (lz4.c:1707-1729): error only if no room at the
             * start; running into the guard zone just stops accumulating */
            if (ip >= iend - 15) return (int)(-ip - 1);
            unsigned s;
            do {
                s = src[ip++];
                lit += s;
                if (ip >= iend - 15) break;
            } while (s == 255);
        }
        if (op + lit > oend - LZ4O_MFLIMIT || ip + lit > iend - 8) {
            /* must be the last sequence: consume the input exactly, fit the output */
            if (ip + lit != iend || op + lit > oend) return (int)(-ip - 1);
            memmove(dst + op, src + ip, (size_t)lit);
            op += lit;
            break;
        }
        memcpy(dst + op, src + ip, (size_t)lit);
        ip += lit;
        op += lit;

        int64_t off = (int64_t)src[ip] | ((int64_t)src[ip + 1] << 8);
        ip += 2;
        int64_t ml = tok & 15;
        if (ml == 15) {
            unsigned s;
            do {
                s = src[ip++];
                ml += s;
                if (ip >= iend - LZ4O_LASTLITERALS + 1) return (int)(-ip - 1);
            } while (s == 255);
        }
        ml += LZ4O_MINMATCH;
        if (off > op + prefix) return (int)(-ip - 1);        /* offset before block (or prefix) start */
        if (op + ml > oend - LZ4O_LASTLITERALS) return (int)(-ip - 1);  /* last 5 bytes are literals */
        if (off == 0) { memset(dst + op, 0, (size_t)ml); op += ml; continue; }
        /* forward byte copy reproduces overlapping-match (offset < length) semantics */
        for (int64_t k = 0; k < ml; k++) dst[op + k] = dst[op - off + k];
        op += ml;
    }
    return (int)op;
}
