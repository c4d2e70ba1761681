/*
 * include/lzbench_hip.h -- C-ABI of liblzbench_hip.so, the MI355X (gfx950) drop-in for the
 * lzbench chunk-loop hot path (LZ4 block + snappy raw codecs, bit-exact with the reference
 * lz4 1.9.3 / snappy 1.1.8).  Plain pointers and sizes only.
 *
 * Three layers:
 *
 *  1. lzbench rows -- the exact compressor_desc_t function-pointer signatures of
 *     /root/reference/_lzbench/lzbench.h:113-115, so a maintainer adds rows to comp_desc[]
 *     (lzbench.h:140-219) next to the CUDA rows (lzbench.h:217-218) under BENCH_HAS_HIP:
 *       compress_func   int64_t (*)(char *in, size_t insize, char *out, size_t outsize,
 *                                   size_t level, size_t param2, char *workmem)
 *       init_func       char* (*)(size_t chunk_size, size_t level, size_t ngpus)
 *       deinit_func     void (*)(char *workmem)
 *     Replaces: lzbench_lz4_compress / lzbench_lz4fast_compress / lzbench_lz4_decompress
 *     (compressors.cpp:343-362), lzbench_snappy_compress / _decompress (compressors.cpp:1282-1292),
 *     lzbench_cuda_{init,deinit,memcpy,return_0} and lzbench_nvcomp_* (compressors.cpp:1813-2014).
 *     Error conventions are lzbench's (lzbench.cpp:284-288, :321): compress returns the
 *     compressed length, <= 0 on failure (driver then stores raw); decompress returns the
 *     decompressed length, <= 0 on error.
 *
 *  2. batched rows -- one call per chunk list instead of one per chunk (the per-chunk ABI
 *     serialises a GPU); replaces the two chunk loops
 *     lzbench_compress / lzbench_decompress (lzbench.cpp:266-298 / :301-329) including the
 *     raw-store rule (clen <= 0 || clen == part -> stored raw, compr_size = part) and the
 *     contiguous packing in chunk order.  Chunks are sharded over the GPUs given to init
 *     (param2 = ngpus): the chunk list is cut into ~128 MiB sub-batches of consecutive chunks,
 *     dealt round-robin to the devices (each pipelines copy-in / kernels / copy-out on its own
 *     streams), and one host-side gather copies every sub-batch's packed bytes to its chunk-order
 *     offset as soon as its sizes land -- so no device's copy-out waits for the devices before it
 *     to finish their whole share.  (One process per GPU under torchrun instead gives each rank
 *     one contiguous slab, lzbench_amd/shard.py)
 *
 *  3. device-resident API -- inputs already in HBM, asynchronous on a caller stream
 *     (the nvcomp batched API analogue, reference nvcomp/lz4.h:239-371).  The input is n
 *     bytes cut into ceil(n/chunk_size) chunks of chunk_size (last one ragged).
 *     Readable-size arguments give how many bytes past the start may be read (>= n + 16):
 *     kernels read whole dwords and rely on that slack.
 */
#ifndef LZBENCH_HIP_H
#define LZBENCH_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* LZH_CODEC_ZSTD: zstd 1.5.2 frames as lzbench's zstd rows write them, one frame per chunk
 * (ZSTD_getParams(level, chunk, 0) + content size, no dictionary, no checksum).  Compression:
 * the fast-strategy levels (zstd 1, 2 where fast, zstd_fast -1..-5), bit-exact with the reference;
 * other levels return LZH_EARG.  Decoding: any frame of that shape, also with the XXH64 content
 * checksum (verified); dictionary ids, a missing content size or windows over 2^27 report -2. */
/* LZH_CODEC_LZ4F: one LZ4 frame per chunk as LZ4F_compressFrame writes it (lz4/lz4frame.c:429-470)
 * with independent blocks, or linked blocks with LZH_LZ4F_LINKED (LZ4_compress_fast_continue in prefix
 * mode, lz4.c:1565-1628); level = LZH_LZ4F_PARAMS(blockSizeID 0|4..7, flags, acceleration).
 * Decoding: frames with independent or linked blocks, every block but the last full, no dictionary id;
 * other frames report -2.
 * LZH_CODEC_NVLZ4: one nvcomp LZ4 container per chunk (the format of the reference's nvcomp_lz4
 * row, nvcomp/LZ4Metadata.h), LZ4 blocks of 1 << (15 + level) bytes, level 0..5 (compressors.cpp:1863).
 * Both: lzh_compress_async / lzh_decompress_async and the rows below; not lzh_compress_kernel_only /
 * lzh_compress_finish_async. */
enum { LZH_CODEC_LZ4 = 0, LZH_CODEC_SNAPPY = 1, LZH_CODEC_MEMCPY = 2, LZH_CODEC_ZSTD = 3, LZH_CODEC_LZ4F = 4,
       LZH_CODEC_NVLZ4 = 5 };
#define LZH_LZ4F_BLOCK_CHECKSUM   0x10   /* LZ4F_blockChecksumEnabled */
#define LZH_LZ4F_CONTENT_CHECKSUM 0x20   /* LZ4F_contentChecksumEnabled */
#define LZH_LZ4F_CONTENT_SIZE     0x40   /* frameInfo.contentSize = chunk size */
#define LZH_LZ4F_LINKED           0x80   /* LZ4F_blockLinked (the LZ4F default; frames of one block stay independent) */
#define LZH_LZ4F_PARAMS(bsid, flags, acc) ((bsid) | (flags) | ((acc) << 8))
enum { LZH_OK = 0, LZH_EARG = -1, LZH_EHIP = -2, LZH_ESPACE = -3, LZH_ECORRUPT = -4 };

/* ---- 1. lzbench rows (per-chunk ABI) ------------------------------------------------ */
char*   lzbench_hip_lz4_init(size_t chunk_size, size_t level, size_t ngpus);
char*   lzbench_hip_snappy_init(size_t chunk_size, size_t level, size_t ngpus);
char*   lzbench_hip_memcpy_init(size_t chunk_size, size_t level, size_t ngpus);
char*   lzbench_hip_zstd_init(size_t chunk_size, size_t level, size_t ngpus);
char*   lzbench_hip_lz4frame_init(size_t chunk_size, size_t level, size_t ngpus);
char*   lzbench_hip_nvcomp_lz4_init(size_t chunk_size, size_t level, size_t ngpus);
void    lzbench_hip_deinit(char* workmem);
/* lz4: LZ4_compress_default semantics; lz4fast: level = acceleration (LZ4_compress_fast) */
int64_t lzbench_hip_lz4_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
int64_t lzbench_hip_lz4fast_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
int64_t lzbench_hip_lz4_decompress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
int64_t lzbench_hip_snappy_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
int64_t lzbench_hip_snappy_decompress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
/* zstd: lzbench_zstd_compress / _decompress semantics (compressors.cpp:1745-1778); level as the
 * zstd / zstd_fast rows pass it (size_t of a possibly negative int) */
int64_t lzbench_hip_zstd_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
int64_t lzbench_hip_zstd_decompress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
/* LZ4 frame per chunk: level = LZH_LZ4F_PARAMS(...): 4..7 = blockSizeID 64 KiB .. 4 MiB without flags,
 * e.g. 0x74 = 64 KiB blocks + block / content checksums + content size */
int64_t lzbench_hip_lz4frame_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
int64_t lzbench_hip_lz4frame_decompress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
/* nvcomp LZ4 container per chunk: replaces lzbench_nvcomp_compress / _decompress (compressors.cpp:1916-2014),
 * level 0..5 = chunks of 32 KiB << level */
int64_t lzbench_hip_nvcomp_lz4_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
int64_t lzbench_hip_nvcomp_lz4_decompress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);
/* hipMemcpy plumbing row: host -> HBM -> host round trip of the chunk */
int64_t lzbench_hip_memcpy(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t p2, char* workmem);

/* ---- 2. batched rows ----------------------------------------------------------------- */
/* Compress nchunks consecutive chunks of in (sizes chunk_sizes[]) into out (capacity
 * outcap), filling compr_sizes[]; applies the raw-store rule. Returns total packed bytes,
 * <= 0 on failure.  The codec and level come from the init call that made workmem. */
int64_t lzbench_hip_compress_batch(const char* in, const size_t* chunk_sizes, int nchunks, char* out,
                                   size_t outcap, size_t* compr_sizes, size_t level, size_t p2, char* workmem);
/* Inverse: out receives sum(chunk_sizes) bytes. Returns that total, <= 0 on error. */
int64_t lzbench_hip_decompress_batch(const char* in, const size_t* compr_sizes, const size_t* chunk_sizes,
                                     int nchunks, char* out, size_t outcap, size_t level, size_t p2, char* workmem);

/* ---- 3. device-resident API ---------------------------------------------------------- */
/* bytes of the per-chunk staging slot (>= worst-case compressed chunk, 256-aligned) */
size_t lzh_stage_stride(int codec, size_t chunk_size);
/* upper bound of the packed output for n bytes */
size_t lzh_max_packed_bytes(int codec, size_t n, size_t chunk_size);
size_t lzh_compress_temp_bytes(int codec, size_t n, size_t chunk_size);
size_t lzh_decompress_temp_bytes(int codec, size_t n, size_t chunk_size);
size_t lzh_num_chunks(size_t n, size_t chunk_size);
/* 1 when the GPU codec compresses at `level` for chunks of up to chunk_size bytes, else 0 (the
 * rows and lzh_compress_async then return LZH_EARG): zstd at the levels whose ZSTD_getParams row
 * is the fast strategy for every chunk size up to chunk_size (lzbench's zstd level 2 is double-fast
 * above 256 KiB: compressors.cpp:1752 via clevels.h); LZ4F / nvcomp at the parameters above. */
int lzh_level_supported(int codec, int level, size_t chunk_size);
/* The batched rows' sharding plan (api.cpp make_plan) and per-shard buffer sizes for n bytes in
 * chunks of chunk_size over ngpus shards, into out[0 .. nout): chunks, chunks per sub-batch,
 * sub-batches, shards, compress input / packed / temp bytes per sub-batch slot, then the sub-batch
 * slots of shard 0 .. shards-1.  Host arithmetic only (no device call).  Returns the count written. */
int lzh_debug_plan(size_t ngpus, size_t n, size_t chunk_size, int codec, uint64_t* out, int nout);
/* The batched rows' host gather order (api.cpp GatherOrder): sub-batches 0 .. nsb-1 complete in
 * `order` (a permutation) with packed sizes sizes[j]; placed[3i .. 3i+2] = (sub-batch, output offset,
 * index into `order` of the completion that made it placeable) for the i-th placement.  Host
 * arithmetic only.  Returns the number of placements (nsb). */
int lzh_debug_gather_order(size_t nsb, const uint64_t* order, const uint64_t* sizes, uint64_t* placed);

/* d_csizes: nchunks u32 (out); d_offsets: nchunks+1 u64 (out; [nchunks] = packed total).
 * level: lz4 acceleration (<=1 -> LZ4_compress_default); zstd level; ignored by snappy. */
int lzh_compress_async(int codec, int level, const void* d_in, size_t n, size_t in_readable, size_t chunk_size,
                       void* d_packed, size_t packed_cap, uint32_t* d_csizes, uint64_t* d_offsets,
                       void* d_temp, size_t temp_bytes, void* hip_stream);
/* d_offsets may be NULL (then derived from d_csizes into d_temp).  d_temp / temp_bytes: LZ4 uses temp only
 * for those derived offsets; LZ4 frames / nvcomp need lzh_decompress_temp_bytes; zstd runs its
 * four-kernel decoder in temp when temp_bytes >= lzh_decompress_temp_bytes (chunks of 16 KiB and more),
 * else every frame in the one-wave decoder (same results, slower); snappy chunks of 512 KiB .. 4 MiB
 * (8..64 fragments of 64 KiB) decode a fragment per wave (split at the tag that starts each fragment,
 * whole where that is not possible) when temp_bytes >= lzh_decompress_temp_bytes, else whole (same
 * results, slower).  d_status: nchunks i32,
 * decoded size per chunk or negative on malformed input (zstd / LZ4 frame / nvcomp container:
 * -1 corrupt, -2 unsupported frame feature).  A chunk whose compressed size equals its size is stored raw (all codecs).
 * Replaces (zstd): lzbench_zstd_decompress, compressors.cpp:1767-1773 (ZSTD_decompressDCtx). */
int lzh_decompress_async(int codec, const void* d_packed, size_t packed_readable, const uint32_t* d_csizes,
                         const uint64_t* d_offsets, size_t n, size_t chunk_size, void* d_out, int32_t* d_status,
                         void* d_temp, size_t temp_bytes, void* hip_stream);

/* Dispatch the stages of lzh_compress_async separately (profiling / roofline): the codec
 * kernel alone writes the staging slots and per-chunk sizes. */
int lzh_compress_kernel_only(int codec, int level, const void* d_in, size_t n, size_t in_readable,
                             size_t chunk_size, void* d_stage, uint32_t* d_csizes, void* hip_stream);

/* One stage of lzh_compress_kernel_only (profiling, roofline of one kernel): stage_mask bit 0 =
 * the parse kernel (LZ4 / snappy: sequence records, chunks up to 16 MiB; zstd: the whole codec),
 * bit 1 = the LZ4 / snappy block-emission kernel (records -> staging slots and sizes).  Both
 * bits = lzh_compress_kernel_only. */
int lzh_compress_kernel_stage(int codec, int level, int stage_mask, const void* d_in, size_t n, size_t in_readable,
                              size_t chunk_size, void* d_stage, uint32_t* d_csizes, void* hip_stream);

/* The rest of lzh_compress_async after lzh_compress_kernel_only: scan the per-chunk sizes
 * into d_offsets and pack the staged streams (or the raw input) into d_packed. */
int lzh_compress_finish_async(int codec, const void* d_in, size_t n, size_t in_readable, size_t chunk_size,
                              const void* d_stage, const uint32_t* d_csizes, void* d_packed, size_t packed_cap,
                              uint64_t* d_offsets, void* hip_stream);

/* synthetic corpora of SURVEY.md 8(d): 0 random, 1 text, 2 json logs, 3 mixed, 4 binary */
size_t lzh_datagen(int kind, uint64_t seed, void* buf, size_t n);
const char* lzh_version(void);

#ifdef __cplusplus
}
#endif
#endif
