/*
 * lzbench_amd/csrc/datagen.c -- deterministic synthetic corpora for the bench and tests
 * (SURVEY.md section 8(d)): enwik8 / Silesia are not available offline, so the configs of
 * BASELINE.json run on these stand-ins.
 *
 *   LZB_DATA_RANDOM  uniform bytes, splitmix64(seed)
 *   LZB_DATA_TEXT    lines of 12 words drawn Zipf(s=1) from a fixed 5000-word vocabulary
 *                    (word length 2..10, a..z)
 *   LZB_DATA_JSON    JSON log lines {"ts","level","svc","req","lat_ms","msg"}: monotone ts,
 *                    4 levels, 5 services, 32-bit request id, exponential latency
 *   LZB_DATA_MIXED   64 MiB stripes cycling text, json, binary counters+noise, random
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>

enum { LZB_DATA_RANDOM = 0, LZB_DATA_TEXT = 1, LZB_DATA_JSON = 2, LZB_DATA_MIXED = 3, LZB_DATA_BINARY = 4 };

typedef struct { uint64_t s; } sm64;
static uint64_t sm_next(sm64* r) {
    uint64_t z = (r->s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double sm_unit(sm64* r) { return (double)(sm_next(r) >> 11) * (1.0 / 9007199254740992.0); }

#define VOCAB 5000
#define ZIPF_LUT_BITS 20
typedef struct {
    char words[VOCAB][11];
    uint8_t lens[VOCAB];
    double cdf[VOCAB];
    uint16_t lut[1 << ZIPF_LUT_BITS];   /* inverse CDF quantised to 2^20 buckets */
} vocab_t;

static void vocab_init(vocab_t* v, uint64_t seed) {
    sm64 r = { seed ^ 0x5eedf00dull };
    double acc = 0;
    for (int i = 0; i < VOCAB; i++) {
        int len = 2 + (int)(sm_next(&r) % 9);
        for (int k = 0; k < len; k++) v->words[i][k] = (char)('a' + sm_next(&r) % 26);
        v->words[i][len] = 0;
        v->lens[i] = (uint8_t)len;
        acc += 1.0 / (double)(i + 1);
        v->cdf[i] = acc;
    }
    for (int i = 0; i < VOCAB; i++) v->cdf[i] /= acc;
    int w = 0;
    for (int b = 0; b < (1 << ZIPF_LUT_BITS); b++) {
        double u = ((double)b + 0.5) / (double)(1 << ZIPF_LUT_BITS);
        while (w < VOCAB - 1 && v->cdf[w] < u) w++;
        v->lut[b] = (uint16_t)w;
    }
}

static int vocab_pick(const vocab_t* v, sm64* r) {
    return v->lut[sm_next(r) >> (64 - ZIPF_LUT_BITS)];
}

static size_t gen_random(uint8_t* buf, size_t n, uint64_t seed) {
    sm64 r = { seed };
    size_t i = 0;
    for (; i + 8 <= n; i += 8) { uint64_t x = sm_next(&r); memcpy(buf + i, &x, 8); }
    if (i < n) { uint64_t x = sm_next(&r); memcpy(buf + i, &x, n - i); }
    return n;
}

static size_t gen_text(uint8_t* buf, size_t n, uint64_t seed, const vocab_t* v) {
    sm64 r = { seed };
    size_t op = 0;
    char line[160];
    while (op < n) {
        int lp = 0;
        for (int w = 0; w < 12; w++) {
            int id = vocab_pick(v, &r);
            memcpy(line + lp, v->words[id], v->lens[id]);
            lp += v->lens[id];
            line[lp++] = (w == 11) ? '\n' : ' ';
        }
        size_t take = (size_t)lp < n - op ? (size_t)lp : n - op;
        memcpy(buf + op, line, take);
        op += take;
    }
    return n;
}

static size_t gen_json(uint8_t* buf, size_t n, uint64_t seed, const vocab_t* v) {
    static const char* levels[4] = { "DEBUG", "INFO", "WARN", "ERROR" };
    static const char* svcs[5] = { "auth", "billing", "search", "gateway", "storage" };
    static const char* verbs[8] = { "request served", "cache miss", "retrying upstream", "user login ok",
                                    "token refreshed", "slow query", "connection reset", "payload accepted" };
    sm64 r = { seed };
    uint64_t ts = 1700000000000ull;
    size_t op = 0;
    char line[320];
    while (op < n) {
        ts += sm_next(&r) % 50;
        uint64_t x = sm_next(&r);
        int lvl = (int)(x % 100);
        lvl = lvl < 10 ? 0 : (lvl < 80 ? 1 : (lvl < 95 ? 2 : 3));
        double lat = -log(1.0 - sm_unit(&r)) * 20.0;
        int a = vocab_pick(v, &r), b = vocab_pick(v, &r);
        int lp = snprintf(line, sizeof line,
                          "{\"ts\":%llu,\"level\":\"%s\",\"svc\":\"%s\",\"req\":\"%08x\",\"lat_ms\":%.3f,"
                          "\"msg\":\"%s %s %s\"}\n",
                          (unsigned long long)ts, levels[lvl], svcs[(x >> 8) % 5], (unsigned)(x >> 32), lat,
                          verbs[(x >> 16) % 8], v->words[a], v->words[b]);
        size_t take = (size_t)lp < n - op ? (size_t)lp : n - op;
        memcpy(buf + op, line, take);
        op += take;
    }
    return n;
}

static size_t gen_binary(uint8_t* buf, size_t n, uint64_t seed) {
    sm64 r = { seed };
    uint32_t ctr[4] = { 0, 1000, 1u << 20, 7 };
    size_t op = 0;
    while (op < n) {
        uint64_t x = sm_next(&r);
        int k = (int)(x & 3);
        ctr[k] += 1 + (uint32_t)((x >> 8) & 3);
        uint32_t w = (x >> 16) % 16 == 0 ? (uint32_t)(x >> 32) : ctr[k];    /* 1/16 noise words */
        size_t take = n - op < 4 ? n - op : 4;
        memcpy(buf + op, &w, take);
        op += take;
    }
    return n;
}

static vocab_t g_vocab;
static pthread_once_t g_vocab_once = PTHREAD_ONCE_INIT;
static void vocab_once(void) { vocab_init(&g_vocab, 12345); }

static size_t gen_one(int kind, uint64_t seed, uint8_t* buf, size_t n) {
    switch (kind) {
    case LZB_DATA_RANDOM: return gen_random(buf, n, seed);
    case LZB_DATA_TEXT: return gen_text(buf, n, seed, &g_vocab);
    case LZB_DATA_JSON: return gen_json(buf, n, seed, &g_vocab);
    case LZB_DATA_BINARY: return gen_binary(buf, n, seed);
    default: return 0;
    }
}

/* Corpora are generated in independent 16 MiB segments (segment s seeded with
 * seed * 1000003 + s), so the bytes do not depend on how many threads produce them. */
#define SEG ((size_t)16 << 20)
typedef struct { int kind; uint64_t seed; uint8_t* buf; size_t off, end, s0, s1; } seg_job;

static int kind_of_segment(int kind, size_t s) {
    static const int order[4] = { LZB_DATA_TEXT, LZB_DATA_JSON, LZB_DATA_BINARY, LZB_DATA_RANDOM };
    if (kind != LZB_DATA_MIXED) return kind;
    return order[(s * SEG / ((size_t)64 << 20)) % 4];     /* 64 MiB stripes */
}

/* segments [s0, s1) of the corpus into buf, which holds corpus bytes [off, end) */
static void* seg_worker(void* a) {
    seg_job* j = (seg_job*)a;
    for (size_t s = j->s0; s < j->s1; s++) {
        size_t pos = s * SEG, len = j->end - pos < SEG ? j->end - pos : SEG;
        gen_one(kind_of_segment(j->kind, s), j->seed * 1000003ull + s, j->buf + (pos - j->off), len);
    }
    return NULL;
}

/* Corpus bytes [off, off + n) of `kind` (off a multiple of 16 MiB: a rank's share of a multi-GiB
 * corpus without generating the bytes before it).  Returns n, or 0 on bad kind / offset. */
size_t lzb_datagen_at(int kind, uint64_t seed, uint8_t* buf, size_t off, size_t n) {
    if (kind < 0 || kind > LZB_DATA_BINARY || off % SEG) return 0;
    pthread_once(&g_vocab_once, vocab_once);
    size_t s0 = off / SEG, nseg = (n + SEG - 1) / SEG;
    int threads = nseg < 16 ? (int)nseg : 16;
    if (threads <= 1) {
        seg_job j = { kind, seed, buf, off, off + n, s0, s0 + nseg };
        seg_worker(&j);
        return n;
    }
    pthread_t th[16];
    seg_job jobs[16];
    for (int t = 0; t < threads; t++) {
        jobs[t] = (seg_job){ kind, seed, buf, off, off + n, s0 + nseg * (size_t)t / (size_t)threads,
                             s0 + nseg * (size_t)(t + 1) / (size_t)threads };
        pthread_create(&th[t], NULL, seg_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    return n;
}

/* Fill buf[0..n) with corpus `kind`. Returns n, or 0 on bad kind. */
size_t lzb_datagen(int kind, uint64_t seed, uint8_t* buf, size_t n) {
    return lzb_datagen_at(kind, seed, buf, 0, n);
}
