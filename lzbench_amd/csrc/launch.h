// lzbench_amd/csrc/launch.h -- host-side launchers exported by each kernel translation unit
// (internal to liblzbench_hip.so; the public C-ABI is include/lzbench_hip.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

hipError_t lzh_launch_lz4_compress_v2(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                      int acc, uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks,
                                      hipStream_t s);
hipError_t lzh_launch_snappy_compress_v2(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                         uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks,
                                         hipStream_t s);
// desc: 32-byte block descriptors (frame_hip.hip) instead of chunk geometry + offsets / csizes
hipError_t lzh_launch_decompress(int codec, const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                                 const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint8_t* out,
                                 int32_t* status, uint32_t nchunks, hipStream_t s, const void* desc = nullptr);
hipError_t lzh_launch_zstd_decompress(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                                      const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint8_t* out,
                                      int32_t* status, uint32_t nchunks, uint8_t* zt, hipStream_t s);
size_t lzh_zstd_decode_temp(uint64_t n, uint64_t chunk_size);
// side stream k (0 or 1; highest priority, created once) of the caller's stream s and its fork / join events
// (decode_hip.hip): work forked to it after a record of `fork` on s joins back through `join`.  False (launch
// on s) when s belongs to another device than the current one.
bool lzh_side_stream(hipStream_t s, hipStream_t& ss, hipEvent_t& fork, hipEvent_t& join, int k = 0);
// snappy chunks of more than one 64 KiB fragment: split scan, fragments in parallel, serial fallback
size_t lzh_snappy_split_temp(uint64_t n, uint64_t chunk_size);
hipError_t lzh_launch_snappy_split_decompress(const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                                              const uint32_t* csizes, uint64_t n_total, uint64_t chunk_size, uint8_t* out,
                                              int32_t* status, uint32_t nchunks, uint8_t* temp, hipStream_t s);
// smallest chunk the zstd split decoder takes (below it: the one-wave decoder, no temp)
constexpr uint64_t lzh_zstd_split_min = 16384;
hipError_t lzh_launch_scan(const uint32_t* csizes, uint64_t nchunks, uint64_t* offsets, uint64_t* total,
                           hipStream_t s);
hipError_t lzh_launch_pack(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                           const uint8_t* stage, uint64_t stride, const uint32_t* csizes, const uint64_t* offsets,
                           uint8_t* packed, uint64_t packed_cap, uint32_t nchunks, hipStream_t s);
hipError_t lzh_launch_memcpy(const void* src, void* dst, uint64_t n, hipStream_t s);
hipError_t lzh_launch_zstd_compress(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                    int level, uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks,
                                    uint8_t* scratch, hipStream_t s);
size_t lzh_zstd_scratch_stride(size_t chunk_size, int level);
int lzh_zstd_level_ok(int level, size_t chunk_size);
// frame_size / bpf: framed layouts (LZ4 frame, nvcomp container) -- block i is block i mod bpf of
// frame i / bpf (frames of frame_size bytes cut into blocks of chunk_size); bpf <= 1: plain chunks
hipError_t lzh_launch_lz4f_linked(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t fs, uint64_t bs,
                                  uint32_t bpf, int acc, uint8_t* stage, uint64_t stride, uint32_t* bcs, uint32_t* snap,
                                  uint32_t nframes, hipStream_t s);
hipError_t lzh_launch_lz4_split(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size, int acc,
                                uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks, uint8_t* recs,
                                int stage_mask, hipStream_t s, uint64_t frame_size = 0, uint32_t bpf = 1);
size_t lzh_lz4_rec_stride(uint64_t chunk_size);
hipError_t lzh_launch_snappy_split(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                                   uint8_t* stage, uint64_t stride, uint32_t* csizes, uint32_t nchunks, uint8_t* recs,
                                   int stage_mask, hipStream_t s);
size_t lzh_snappy_rec_stride(uint64_t chunk_size);
uint32_t lzh_snappy_frags(uint64_t chunk_size);

// framed LZ4 layouts (frame_hip.hip); codec 4 = LZ4 frame, 5 = nvcomp LZ4 container
hipError_t lzh_launch_frame_sizes(int codec, int params, uint64_t n_total, uint64_t fs, uint64_t bs, uint32_t bpf,
                                  const uint32_t* bcs, uint32_t* rel, uint32_t* csizes, uint32_t nframes, hipStream_t s);
hipError_t lzh_launch_frame_pack(int codec, int params, const uint8_t* in, uint64_t n_total, uint64_t in_readable,
                                 uint64_t fs, uint64_t bs, uint32_t bpf, const uint8_t* stage, uint64_t stride,
                                 const uint32_t* bcs, const uint32_t* rel, const uint32_t* csizes,
                                 const uint64_t* offsets, uint8_t* packed, uint32_t nblocks, uint32_t nframes,
                                 hipStream_t s);
hipError_t lzh_launch_frame_parse(int codec, const uint8_t* packed, uint64_t packed_readable, const uint64_t* offsets,
                                  const uint32_t* csizes, uint64_t n_total, uint64_t fs, uint32_t maxbpf, void* desc,
                                  int32_t* fstat, uint32_t nframes, hipStream_t s);
hipError_t lzh_launch_frame_finish(int codec, const uint8_t* packed, const uint64_t* offsets, const uint32_t* csizes,
                                   uint64_t n_total, uint64_t fs, uint32_t maxbpf, const void* desc,
                                   const int32_t* bstat, const int32_t* fstat, const uint8_t* out, int32_t* status,
                                   uint32_t nframes, hipStream_t s);
