/*
 * oracle/chunks_oracle.c -- the lzbench chunk loop restated in C.  TEST INFRASTRUCTURE ONLY.
 *
 *   lzbench_compress   /root/reference/_lzbench/lzbench.cpp:266-298
 *     per chunk: clen = compress(...); if (clen <= 0 || clen == part) store raw;
 *     outputs packed back to back, compr_sizes[i] = clen.
 *   lzbench_decompress /root/reference/_lzbench/lzbench.cpp:301-329
 *     per chunk: if (compr_size == chunk_size) memcpy else decompress; stop on dlen <= 0.
 *
 * The _mt variants split the same chunk list over pthreads (each thread compresses its
 * contiguous chunk range into a private staging area, then ranges are packed in order),
 * giving the "all host cores" CPU baseline of SURVEY.md section 8(d).
 */
#include "oracle.h"
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

static int64_t compress_one(int codec, int level, const uint8_t* in, size_t part, uint8_t* out) {
    if (codec == 2) return oracle_zstd_compress(in, part, out, level);
    if (codec == 3) return oracle_lz4f_compress(in, part, out, level);
    if (codec == 4) return oracle_nvlz4_compress(in, part, out, level);
    if (codec == 0) return oracle_lz4_compress(in, (int)part, out, level < 1 ? 1 : level);
    return (int64_t)oracle_snappy_compress(in, part, out);
}

static size_t bound_one(int codec, size_t part) {
    if (codec == 2) return oracle_zstd_bound(part) + 64;
    if (codec == 3) return oracle_lz4f_bound(part, 4);   /* (64 KiB blocks: the most block words, raw at worst) */
    if (codec == 4) return oracle_nvlz4_bound(part, 0);
    return codec == 0 ? (size_t)oracle_lz4_bound((int)part) : oracle_snappy_bound(part);
}

static int64_t decompress_one(int codec, const uint8_t* in, size_t csize, uint8_t* out, size_t cap) {
    if (codec == 2) return -1;   /* zstd decoding: the reference build is the checker */
    if (codec == 3) return oracle_lz4f_decompress(in, csize, out, cap);
    if (codec == 4) return oracle_nvlz4_decompress(in, csize, out, cap);
    if (codec == 0) return oracle_lz4_decompress_safe(in, (int)csize, out, (int)cap);
    return oracle_snappy_uncompress(in, csize, out, cap);
}

int64_t oracle_compress_chunks(int codec, int level, const uint8_t* in, size_t n,
                               size_t chunk_size, uint8_t* out, uint64_t* csizes) {
    size_t nchunks = (n + chunk_size - 1) / chunk_size;
    size_t maxb = bound_one(codec, chunk_size);
    uint8_t* tmp = (uint8_t*)malloc(maxb + 64);
    int64_t sum = 0;
    for (size_t i = 0; i < nchunks; i++) {
        size_t part = (i + 1 < nchunks) ? chunk_size : n - i * chunk_size;
        int64_t clen = compress_one(codec, level, in + i * chunk_size, part, tmp);
        if (clen <= 0 || (size_t)clen == part) { memcpy(out + sum, in + i * chunk_size, part); clen = (int64_t)part; }
        else memcpy(out + sum, tmp, (size_t)clen);
        csizes[i] = (uint64_t)clen;
        sum += clen;
    }
    free(tmp);
    return sum;
}

int64_t oracle_decompress_chunks(int codec, const uint8_t* packed, const uint64_t* csizes,
                                 size_t n, size_t chunk_size, uint8_t* out) {
    size_t nchunks = (n + chunk_size - 1) / chunk_size;
    size_t ip = 0;
    int64_t sum = 0;
    for (size_t i = 0; i < nchunks; i++) {
        size_t part = (i + 1 < nchunks) ? chunk_size : n - i * chunk_size;
        int64_t dlen;
        if (csizes[i] == part) { memcpy(out + i * chunk_size, packed + ip, part); dlen = (int64_t)part; }
        else dlen = decompress_one(codec, packed + ip, csizes[i], out + i * chunk_size, part);
        if (dlen <= 0) return dlen;
        ip += csizes[i];
        sum += dlen;
    }
    return sum;
}

typedef struct {
    int codec, level;
    const uint8_t* in;
    size_t n, chunk_size, c0, c1;
    uint8_t* out;          /* compress: private staging; decompress: final output */
    const uint8_t* packed;
    uint64_t* csizes;
    const uint64_t* offsets;
    int64_t result;
} mt_job;

static void* mt_compress_worker(void* arg) {
    mt_job* j = (mt_job*)arg;
    size_t nchunks = (j->n + j->chunk_size - 1) / j->chunk_size;
    size_t maxb = bound_one(j->codec, j->chunk_size);
    uint8_t* tmp = (uint8_t*)malloc(maxb + 64);
    int64_t sum = 0;
    for (size_t i = j->c0; i < j->c1; i++) {
        size_t part = (i + 1 < nchunks) ? j->chunk_size : j->n - i * j->chunk_size;
        const uint8_t* src = j->in + i * j->chunk_size;
        int64_t clen = compress_one(j->codec, j->level, src, part, tmp);
        if (clen <= 0 || (size_t)clen == part) { memcpy(j->out + sum, src, part); clen = (int64_t)part; }
        else memcpy(j->out + sum, tmp, (size_t)clen);
        j->csizes[i] = (uint64_t)clen;
        sum += clen;
    }
    free(tmp);
    j->result = sum;
    return NULL;
}

int64_t oracle_compress_chunks_mt(int codec, int level, const uint8_t* in, size_t n,
                                  size_t chunk_size, uint8_t* out, uint64_t* csizes, int threads) {
    size_t nchunks = (n + chunk_size - 1) / chunk_size;
    if (threads < 1) threads = 1;
    if ((size_t)threads > nchunks) threads = nchunks ? (int)nchunks : 1;
    mt_job* jobs = (mt_job*)calloc((size_t)threads, sizeof(mt_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    size_t maxb = bound_one(codec, chunk_size);
    for (int t = 0; t < threads; t++) {
        mt_job* j = &jobs[t];
        j->codec = codec; j->level = level; j->in = in; j->n = n; j->chunk_size = chunk_size;
        j->c0 = nchunks * (size_t)t / (size_t)threads;
        j->c1 = nchunks * (size_t)(t + 1) / (size_t)threads;
        j->csizes = csizes;
        j->out = (uint8_t*)malloc((j->c1 - j->c0) * (maxb > chunk_size ? maxb : chunk_size) + 64);
        pthread_create(&th[t], NULL, mt_compress_worker, j);
    }
    int64_t sum = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        memcpy(out + sum, jobs[t].out, (size_t)jobs[t].result);   /* host-side gather in chunk order */
        sum += jobs[t].result;
        free(jobs[t].out);
    }
    free(jobs); free(th);
    return sum;
}

static void* mt_decompress_worker(void* arg) {
    mt_job* j = (mt_job*)arg;
    size_t nchunks = (j->n + j->chunk_size - 1) / j->chunk_size;
    int64_t sum = 0;
    for (size_t i = j->c0; i < j->c1; i++) {
        size_t part = (i + 1 < nchunks) ? j->chunk_size : j->n - i * j->chunk_size;
        const uint8_t* src = j->packed + j->offsets[i];
        int64_t dlen;
        if (j->csizes[i] == part) { memcpy(j->out + i * j->chunk_size, src, part); dlen = (int64_t)part; }
        else dlen = decompress_one(j->codec, src, j->csizes[i], j->out + i * j->chunk_size, part);
        if (dlen <= 0) { j->result = dlen; return NULL; }
        sum += dlen;
    }
    j->result = sum;
    return NULL;
}

int64_t oracle_decompress_chunks_mt(int codec, const uint8_t* packed, const uint64_t* csizes,
                                    size_t n, size_t chunk_size, uint8_t* out, int threads) {
    size_t nchunks = (n + chunk_size - 1) / chunk_size;
    if (threads < 1) threads = 1;
    if ((size_t)threads > nchunks) threads = nchunks ? (int)nchunks : 1;
    uint64_t* offs = (uint64_t*)malloc((nchunks + 1) * sizeof(uint64_t));
    offs[0] = 0;
    for (size_t i = 0; i < nchunks; i++) offs[i + 1] = offs[i] + csizes[i];
    mt_job* jobs = (mt_job*)calloc((size_t)threads, sizeof(mt_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    for (int t = 0; t < threads; t++) {
        mt_job* j = &jobs[t];
        j->codec = codec; j->n = n; j->chunk_size = chunk_size; j->packed = packed;
        j->csizes = (uint64_t*)csizes; j->offsets = offs; j->out = out;
        j->c0 = nchunks * (size_t)t / (size_t)threads;
        j->c1 = nchunks * (size_t)(t + 1) / (size_t)threads;
        pthread_create(&th[t], NULL, mt_decompress_worker, j);
    }
    int64_t sum = 0, err = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(th[t], NULL);
        if (jobs[t].result <= 0 && jobs[t].c1 > jobs[t].c0) err = jobs[t].result ? jobs[t].result : -1;
        sum += jobs[t].result;
    }
    free(jobs); free(th); free(offs);
    return err ? err : sum;
}
