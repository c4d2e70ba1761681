/*
 * oracle/oracle.h -- CPU restatement of the reference codecs on the lzbench hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (lzbench_amd/, include/, the
 * C-ABI library) may include, link or call anything under oracle/.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, and only as the
 * checker / CPU baseline, never as the thing measured on the GPU.
 *
 * Pinning: these restatements are checked byte-for-byte against golden vectors
 * produced by the reference's own lz4 1.9.3 / snappy 1.1.8 sources compiled from
 * /root/reference (oracle/Makefile target `ref`, outputs in oracle/_ref/), see
 * tests/golden/make_golden.py and tests/test_oracle.py.
 */
#ifndef LZB_ORACLE_H
#define LZB_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* LZ4 block compression, LZ4_compress_fast(src,dst,n,cap>=bound,acc) semantics
 * (reference lz4/lz4.c:1284-1305 notLimited path, :851-1240 parser). Returns bytes written. */
int oracle_lz4_compress(const uint8_t* src, int n, uint8_t* dst, int acceleration);
/* LZ4_compressBound (reference lz4/lz4.h:171). */
int oracle_lz4_bound(int n);
/* LZ4_decompress_safe semantics (reference lz4/lz4.c:1737-2165 safe loop, :2170-2176).
 * Returns decoded size, or a negative value on malformed input. */
int oracle_lz4_decompress_safe(const uint8_t* src, int csize, uint8_t* dst, int cap);
int oracle_lz4_decompress_prefix(const uint8_t* src, int csize, uint8_t* dst, int cap, int64_t prefix);

/* snappy::RawCompress (reference snappy/snappy.cc:1043-1111, :510-681). Returns bytes written. */
size_t oracle_snappy_compress(const uint8_t* src, size_t n, uint8_t* dst);
/* snappy::MaxCompressedLength (reference snappy/snappy.cc:99-121). */
size_t oracle_snappy_bound(size_t n);
/* snappy::RawUncompress (reference snappy/snappy.cc:848-1036, :1398-1407).
 * Returns the uncompressed size on success, -1 on malformed input. cap = output capacity. */
int64_t oracle_snappy_uncompress(const uint8_t* src, size_t csize, uint8_t* dst, size_t cap);

/* zstd 1.5.2 frame compression as lzbench's zstd rows call it (ZSTD_getParams(level, n, 0) with
 * contentSizeFlag, ZSTD_compress_advanced; reference _lzbench/compressors.cpp:1745-1770), for the
 * fast-strategy levels (-131072..-1, 1, 2; level 2 only where it is fast).  dst needs
 * oracle_zstd_bound(n) + 64 bytes.  Returns the frame size, or -1 for an unsupported level. */
int64_t oracle_zstd_compress(const uint8_t* src, size_t n, uint8_t* dst, int level);
size_t oracle_zstd_bound(size_t n);

/* Framed LZ4 formats (frame_oracle.c).  LZ4 frame as LZ4F_compressFrame writes it with
 * independent blocks (lz4frame.c:373-1019); params: bits 0-2 blockSizeID (0 = default 64 KiB, 4..7),
 * 0x10 block checksum, 0x20 content checksum, 0x40 content size, bits 8-15 acceleration.
 * nvcomp LZ4 container (nvcomp/LZ4Metadata.h): chunks of 1 << (15 + level) bytes, LZ4 blocks.
 * Decoders return the decoded size, -1 on malformed input, -2 for an unsupported feature. */
uint32_t oracle_xxh32(const uint8_t* p, size_t len, uint32_t seed);
size_t  oracle_lz4f_bound(size_t n, int params);
int64_t oracle_lz4f_compress(const uint8_t* src, size_t n, uint8_t* dst, int params);
int64_t oracle_lz4f_decompress(const uint8_t* src, size_t csize, uint8_t* dst, size_t cap);
size_t  oracle_nvlz4_bound(size_t n, int level);
int64_t oracle_nvlz4_compress(const uint8_t* src, size_t n, uint8_t* dst, int level);
int64_t oracle_nvlz4_decompress(const uint8_t* src, size_t csize, uint8_t* dst, size_t cap);

/* lzbench chunk loop (reference _lzbench/lzbench.cpp:266-298): compress every chunk,
 * store raw when clen<=0 || clen==part, pack contiguously. codec: 0=lz4 1=snappy 2=zstd
 * (compression only) 3=lz4 frame 4=nvcomp lz4 container (level = their params).
 * level: lz4 acceleration (0 or 1 -> default). Returns total packed bytes. */
int64_t oracle_compress_chunks(int codec, int level, const uint8_t* in, size_t n,
                               size_t chunk_size, uint8_t* out, uint64_t* csizes);
/* lzbench_decompress (reference _lzbench/lzbench.cpp:301-329). Returns total or <=0 on error. */
int64_t oracle_decompress_chunks(int codec, const uint8_t* packed, const uint64_t* csizes,
                                 size_t n, size_t chunk_size, uint8_t* out);
/* Same loops over the chunk list split across `threads` pthreads (CPU baseline, all cores). */
int64_t oracle_compress_chunks_mt(int codec, int level, const uint8_t* in, size_t n,
                                  size_t chunk_size, uint8_t* out, uint64_t* csizes, int threads);
int64_t oracle_decompress_chunks_mt(int codec, const uint8_t* packed, const uint64_t* csizes,
                                    size_t n, size_t chunk_size, uint8_t* out, int threads);

#ifdef __cplusplus
}
#endif
#endif
