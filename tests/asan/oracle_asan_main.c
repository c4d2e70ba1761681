/* tests/asan/oracle_asan_main.c -- sanitizer harness for the C code of the repo that runs on the
 * host: the oracle restatements (oracle/*.c) and the corpus generator (lzbench_amd/csrc/datagen.c).
 * Built with -fsanitize=address,undefined by tests/test_sanitizers.py (the
 * reference has no sanitizer runs; the CPU restatement gets them here).  Exit 0 = clean run. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "../../oracle/oracle.h"

size_t lzb_datagen(int kind, uint64_t seed, uint8_t* buf, size_t n);

static int roundtrip(int codec, const uint8_t* in, size_t n, size_t chunk, int level) {
    size_t k = (n + chunk - 1) / chunk;
    uint8_t* packed = (uint8_t*)malloc(n + n / 6 + 16384 + 64 * k + 64);
    uint64_t* cs = (uint64_t*)calloc(k ? k : 1, 8);
    uint8_t* out = (uint8_t*)malloc(n + 64);
    int64_t tot = oracle_compress_chunks(codec, level, in, n, chunk, packed, cs);
    int64_t tot_mt = 0;
    uint8_t* packed2 = (uint8_t*)malloc(n + n / 6 + 16384 + 64 * k + 64);
    uint64_t* cs2 = (uint64_t*)calloc(k ? k : 1, 8);
    tot_mt = oracle_compress_chunks_mt(codec, level, in, n, chunk, packed2, cs2, 3);
    int bad = tot <= 0 || tot != tot_mt || memcmp(packed, packed2, (size_t)tot) != 0;
    if (codec != 2) {   /* (zstd frames are decoded by the reference build, not by the oracle) */
        int64_t d = oracle_decompress_chunks(codec, packed, cs, n, chunk, out);
        bad |= d != (int64_t)n || memcmp(in, out, n) != 0;
        d = oracle_decompress_chunks_mt(codec, packed, cs, n, chunk, out, 3);
        bad |= d != (int64_t)n || memcmp(in, out, n) != 0;
    }
    free(packed); free(packed2); free(cs); free(cs2); free(out);
    return bad;
}

int main(void) {
    const size_t n = 3 * 131072 + 4321;
    uint8_t* buf = (uint8_t*)malloc(n + 64);
    int bad = 0;
    for (int kind = 0; kind < 5; kind++) {
        if (lzb_datagen(kind, 7 + kind, buf, n) != n) return 2;
        bad |= roundtrip(0, buf, n, 65536, 1);
        bad |= roundtrip(0, buf, n, 131072, 1);
        bad |= roundtrip(0, buf, n, 65536, 9);
        bad |= roundtrip(1, buf, n, 65536, 0);
        bad |= roundtrip(1, buf, n, 262144, 0);
        bad |= roundtrip(2, buf, n, 131072, 1);
        bad |= roundtrip(2, buf, n, 262144, 1);
        bad |= roundtrip(2, buf, n, 65536, -3);
        bad |= roundtrip(3, buf, n, 65536, 0);          /* LZ4 frames */
        bad |= roundtrip(3, buf, n, 200000, 0x74);
        bad |= roundtrip(3, buf, n, n, 7 | 0x30);
        bad |= roundtrip(4, buf, n, 65536, 0);          /* nvcomp LZ4 containers */
        bad |= roundtrip(4, buf, n, 300000, 2);
    }
    /* malformed streams must be rejected without reading or writing out of bounds */
    for (int t = 0; t < 2000; t++) {
        uint8_t junk[300], out[5000];
        for (int i = 0; i < 300; i++) junk[i] = (uint8_t)(rand() & 0xff);
        (void)oracle_lz4_decompress_safe(junk, 1 + t % 300, out, (int)sizeof(out));
        (void)oracle_snappy_uncompress(junk, 1 + t % 300, out, sizeof(out));
        if (t & 1) { junk[0] = 0x04; junk[1] = 0x22; junk[2] = 0x4d; junk[3] = 0x18; }   /* LZ4F magic */
        else { memset(junk, 0, 8); junk[0] = 4; }                                         /* nvcomp flag */
        (void)oracle_lz4f_decompress(junk, 1 + t % 300, out, sizeof(out));
        (void)oracle_nvlz4_decompress(junk, 1 + t % 300, out, sizeof(out));
    }
    free(buf);
    printf(bad ? "FAIL\n" : "ok\n");
    return bad;
}
