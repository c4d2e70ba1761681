/*
 * oracle/snappy_oracle.c -- plain-C restatement of snappy 1.1.8 raw (un-framed) format
 * as lzbench drives it.  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Restated from the reference algorithm, not copied:
 *   HashBytes, MaxCompressedLength ....... /root/reference/snappy/snappy.cc:94-121
 *   EmitLiteral / EmitCopy(AtMost64) ..... snappy.cc:342-443
 *   CalculateTableSize / per-fragment reset snappy.cc:457-495, :1043-1111
 *   CompressFragment (16 unrolled probes,
 *     skip>>5 heuristic, post-copy inserts) snappy.cc:510-681
 *   FindMatchLength semantics ............ snappy-internal.h:100-224 (len = common prefix)
 *   tag decoding / validity rules ........ snappy.cc:819-1036, :1319-1407, snappy-internal.h:258-310
 */
#include "oracle.h"
#include <string.h>

static uint32_t rd32(const uint8_t* p) { uint32_t v; memcpy(&v, p, 4); return v; }

size_t oracle_snappy_bound(size_t n) { return 32 + n + n / 6; }

static int log2floor(uint32_t v) { int r = -1; while (v) { v >>= 1; r++; } return r; }

static uint32_t table_size_for(uint32_t n) {
    if (n > (1u << 14)) return 1u << 14;
    if (n < (1u << 8)) return 1u << 8;
    return 2u << log2floor(n - 1);
}

static size_t emit_literal(uint8_t* dst, size_t op, const uint8_t* lit, int len) {
    int n = len - 1;
    if (n < 60) {
        dst[op++] = (uint8_t)(n << 2);
    } else {
        int count = (log2floor((uint32_t)n) >> 3) + 1;   /* 1..4 length bytes */
        dst[op++] = (uint8_t)((59 + count) << 2);
        for (int i = 0; i < count; i++) dst[op++] = (uint8_t)(n >> (8 * i));
    }
    memcpy(dst + op, lit, (size_t)len);
    return op + (size_t)len;
}

static size_t emit_copy_le64(uint8_t* dst, size_t op, uint32_t off, int len) {
    if (len < 12 && off < 2048) {          /* COPY_1: 3-bit len-4, 11-bit offset */
        dst[op++] = (uint8_t)(1 | ((len - 4) << 2) | ((off >> 8) << 5));
        dst[op++] = (uint8_t)(off & 0xff);
    } else {                               /* COPY_2: 6-bit len-1, 16-bit offset */
        dst[op++] = (uint8_t)(2 | ((len - 1) << 2));
        dst[op++] = (uint8_t)(off & 0xff);
        dst[op++] = (uint8_t)(off >> 8);
    }
    return op;
}

static size_t emit_copy(uint8_t* dst, size_t op, uint32_t off, int len) {
    if (len < 12) return emit_copy_le64(dst, op, off, len);
    while (len >= 68) { op = emit_copy_le64(dst, op, off, 64); len -= 64; }
    if (len > 64) { op = emit_copy_le64(dst, op, off, 60); len -= 60; }
    return emit_copy_le64(dst, op, off, len);
}

/* one fragment (<= 64 KiB); offsets are relative to the fragment start */
static size_t compress_fragment(const uint8_t* in, uint32_t n, uint8_t* dst, size_t op, uint16_t* table) {
    const uint32_t tsize = table_size_for(n);
    const int shift = 32 - log2floor(tsize);
    memset(table, 0, tsize * sizeof(uint16_t));

    uint32_t ip = 0, next_emit = 0;
    if (n >= 15) {
        const uint32_t ip_limit = n - 15;
        for (;;) {
            next_emit = ip++;
            uint32_t skip = 32;
            uint32_t cand = 0;
            int found = 0;
            if (ip_limit - ip >= 16 && ip <= ip_limit) {
                for (uint32_t i = 0; i < 16; i++) {          /* unrolled probes, no limit check */
                    uint32_t v = rd32(in + ip + i);
                    uint32_t h = (v * 0x1e35a7bdu) >> shift;
                    cand = table[h];
                    table[h] = (uint16_t)(ip + i);
                    if (rd32(in + cand) == v) {
                        ip += i;
                        found = 1;
                        break;
                    }
                }
                if (!found) { ip += 16; skip += 16; }
            }
            if (!found) {
                for (;;) {
                    uint32_t v = rd32(in + ip);
                    uint32_t h = (v * 0x1e35a7bdu) >> shift;
                    uint32_t step = skip >> 5;
                    skip += step;
                    uint32_t next_ip = ip + step;
                    if (next_ip > ip_limit) { ip = next_emit; goto remainder; }
                    cand = table[h];
                    table[h] = (uint16_t)ip;
                    if (v == rd32(in + cand)) break;
                    ip = next_ip;
                }
            }
            op = emit_literal(dst, op, in + next_emit, (int)(ip - next_emit));
            /* copy loop: keep emitting while the position right after a copy matches */
            for (;;) {
                uint32_t base = ip;
                uint32_t m = 4;
                while (ip + m < n && in[cand + m] == in[ip + m]) m++;
                ip += m;
                op = emit_copy(dst, op, base - cand, (int)m);
                if (ip >= ip_limit) goto remainder;
                uint32_t hm1 = (rd32(in + ip - 1) * 0x1e35a7bdu) >> shift;
                table[hm1] = (uint16_t)(ip - 1);
                uint32_t v = rd32(in + ip);
                uint32_t h = (v * 0x1e35a7bdu) >> shift;
                cand = table[h];
                table[h] = (uint16_t)ip;
                if (v != rd32(in + cand)) break;
            }
        }
    }
remainder:
    if (ip < n) op = emit_literal(dst, op, in + ip, (int)(n - ip));
    return op;
}

size_t oracle_snappy_compress(const uint8_t* src, size_t n, uint8_t* dst) {
    static __thread uint16_t table[1 << 14];
    size_t op = 0;
    uint32_t v = (uint32_t)n;
    while (v >= 128) { dst[op++] = (uint8_t)(v | 128); v >>= 7; }   /* varint32 length */
    dst[op++] = (uint8_t)v;
    for (size_t pos = 0; pos < n; pos += 65536) {
        uint32_t frag = (uint32_t)((n - pos) < 65536 ? (n - pos) : 65536);
        op = compress_fragment(src + pos, frag, dst, op, table);
    }
    return op;
}

int64_t oracle_snappy_uncompress(const uint8_t* src, size_t csize, uint8_t* dst, size_t cap) {
    size_t ip = 0;
    uint64_t ulen = 0;
    int shift = 0;
    for (;;) {                                     /* varint32, at most 5 bytes, no overflow */
        if (ip >= csize || shift >= 32) return -1;
        uint8_t c = src[ip++];
        uint64_t val = c & 0x7f;
        if (shift == 28 && val > 15) return -1;
        ulen |= val << shift;
        if (c < 128) break;
        shift += 7;
    }
    if (ulen > cap) return -1;
    size_t op = 0;
    while (ip < csize) {
        uint8_t c = src[ip++];
        uint32_t kind = c & 3;
        if (kind == 0) {
            size_t len = (c >> 2) + 1u;
            if (len > 60) {
                size_t nb = len - 60;
                if (ip + nb > csize) return -1;
                len = 0;
                for (size_t i = 0; i < nb; i++) len |= (size_t)src[ip + i] << (8 * i);
                len += 1;
                ip += nb;
            }
            if (ip + len > csize || op + len > ulen) return -1;
            memcpy(dst + op, src + ip, len);
            ip += len;
            op += len;
        } else {
            size_t len, off;
            size_t extra = kind == 1 ? 1 : (kind == 2 ? 2 : 4);
            if (ip + extra > csize) return -1;
            if (kind == 1) {
                len = ((c >> 2) & 7) + 4;
                off = ((size_t)(c >> 5) << 8) | src[ip];
            } else {
                len = (c >> 2) + 1u;
                off = 0;
                for (size_t i = 0; i < extra; i++) off |= (size_t)src[ip + i] << (8 * i);
            }
            ip += extra;
            if (off == 0 || off > op || op + len > ulen) return -1;
            for (size_t k = 0; k < len; k++) dst[op + k] = dst[op - off + k];
            op += len;
        }
    }
    return op == ulen ? (int64_t)op : -1;
}
