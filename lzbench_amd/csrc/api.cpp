// lzbench_amd/csrc/api.cpp -- the C-ABI of include/lzbench_hip.h.
//
// Device-resident layer: stage -> scan -> pack for compression, scan -> decode for
// decompression, all asynchronous on the caller's stream.
// Host layer: lzbench rows and batched rows.  A row's workmem is an LzhCtx holding, per GPU,
// a stream and device buffers sized at init for the chunk size (grown on demand).  A batch
// is cut into runs of uniform chunking (lzbench's chunk list is uniform per input file,
// lzbench.cpp:366-373); each run is cut into ~128 MiB sub-batches dealt round-robin to the GPUs
// (make_plan), every GPU pipelines its sub-batches (copy in | kernels | copy out), and the host
// places each sub-batch's packed bytes at its chunk-order offset as soon as the sizes before it
// are known.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include <rocprofiler-sdk-roctx/roctx.h>

#include "../../include/lzbench_hip.h"
#include "launch.h"

// rocprof-visible ranges around each stage's launches (rocprofv3 --marker-trace); a range covers
// the enqueue of the stage on the host, the kernels themselves show in --kernel-trace
struct Range {
    explicit Range(const char* n) { roctxRangePushA(n); }
    ~Range() { roctxRangePop(); }
};

extern "C" size_t lzb_datagen(int kind, uint64_t seed, uint8_t* buf, size_t n);

#define LZH_CHECK(x)                                                                  \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "lzbench_hip: %s failed: %s\n", #x, hipGetErrorString(e_)); \
            return LZH_EHIP;                                                          \
        }                                                                             \
    } while (0)

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// LZ4 chunks up to this size compress in two kernels (parse -> 8-byte sequence records -> emit);
// larger ones (24-bit record fields) in the single kernel that assembles the block itself
static const size_t kLz4SplitMax = (size_t)16 << 20;   // LZ4 / snappy parse + emit split up to this chunk size

extern "C" {

const char* lzh_version(void) { return "lzbench_hip 0.2 (lz4 1.9.3 / snappy 1.1.8 / zstd 1.5.2 fast levels bit-exact, gfx950)"; }

size_t lzh_datagen(int kind, uint64_t seed, void* buf, size_t n) { return lzb_datagen(kind, seed, (uint8_t*)buf, n); }

size_t lzh_num_chunks(size_t n, size_t chunk_size) {
    if (chunk_size == 0) return 0;
    return n == 0 ? 1 : (n + chunk_size - 1) / chunk_size;
}

static bool is_frame(int codec) { return codec == LZH_CODEC_LZ4F || codec == LZH_CODEC_NVLZ4; }

static size_t codec_bound(int codec, size_t part) {
    if (codec == LZH_CODEC_LZ4F)    // raw blocks at worst, 64 KiB blocks the smallest: header, block words, end
        return part + 8 * ((part + 65535) / 65536) + 32;
    if (codec == LZH_CODEC_NVLZ4)   // LZ4 blocks of 32 KiB at the least, 8-byte fields
        return part + part / 255 + 24 * ((part + 32767) / 32768) + 48;
    if (codec == LZH_CODEC_LZ4) return part + part / 255 + 16;     // LZ4_compressBound, lz4.h:171
    if (codec == LZH_CODEC_SNAPPY) return 32 + part + part / 6;    // MaxCompressedLength, snappy.cc:99-121
    if (codec == LZH_CODEC_ZSTD)                                    // ZSTD_COMPRESSBOUND, zstd.h:~210
        return part + (part >> 8) + (part < (128u << 10) ? ((128u << 10) - part) >> 11 : 0);
    return part;
}

size_t lzh_stage_stride(int codec, size_t chunk_size) { return align_up(codec_bound(codec, chunk_size) + 16, 256); }

size_t lzh_max_packed_bytes(int codec, size_t n, size_t chunk_size) {
    size_t k = lzh_num_chunks(n, chunk_size);
    return n + k * (codec_bound(codec, chunk_size) - chunk_size + 8) + 64;
}

// Framed layouts: frames of F bytes (the chunks) cut into blocks of bs = min(F, B) bytes
struct FrameGeo {
    size_t F, bs, nframes, nblocks;
    uint32_t bpf;
};

static size_t frame_block_bytes(int codec, int level) {
    if (codec == LZH_CODEC_LZ4F) { const int id = level & 7; return (size_t)1 << (8 + 2 * (id ? id : 4)); }
    return (size_t)32768 << level;
}

static bool frame_level_ok(int codec, int level) {
    if (codec == LZH_CODEC_LZ4F) { const int id = level & 7; return level >= 0 && level < (1 << 16) && (id == 0 || id >= 4) && !(level & 0x08); }
    return level >= 0 && level <= 5;
}

extern "C" int lzh_level_supported(int codec, int level, size_t chunk_size) {
    if (codec == LZH_CODEC_ZSTD) return lzh_zstd_level_ok(level, chunk_size) ? 1 : 0;
    if (codec == LZH_CODEC_LZ4F || codec == LZH_CODEC_NVLZ4) return frame_level_ok(codec, level) ? 1 : 0;
    return codec >= LZH_CODEC_LZ4 && codec <= LZH_CODEC_MEMCPY ? 1 : 0;
}


static FrameGeo frame_geo(size_t B, size_t n, size_t F) {
    FrameGeo g;
    g.F = F;
    g.bs = std::min(F, B);
    g.bpf = (uint32_t)((F + g.bs - 1) / g.bs);
    g.nframes = lzh_num_chunks(n, F);
    if (n == 0) {
        g.nblocks = 0;
    } else {
        const size_t last = n - (g.nframes - 1) * F;
        g.nblocks = (g.nframes - 1) * g.bpf + (last + g.bs - 1) / g.bs;
    }
    return g;
}

// temp of a framed compression: staging slots | LZ4 sequence records (+ 8 B per block) | block
// sizes | block offsets inside their frame
struct FrameTemp { size_t stride, stage, recs, bcs, rel, total; };
static FrameTemp frame_temp(const FrameGeo& g) {
    FrameTemp t;
    t.stride = lzh_stage_stride(LZH_CODEC_LZ4, g.bs);
    t.stage = 0;
    t.recs = align_up(g.nblocks * t.stride, 256) + 256;
    t.bcs = t.recs + g.nblocks * lzh_lz4_rec_stride(g.bs) + align_up(g.nblocks * 8, 256) + 256;
    t.rel = t.bcs + align_up(g.nblocks * 4, 256) + 256;
    t.total = t.rel + align_up(g.nblocks * 4, 256) + 256;
    return t;
}

static size_t frame_temp_worst(int codec, size_t n, size_t F) {
    size_t t = 0;
    for (int l = 0; l < 6; l++) {
        const size_t B = codec == LZH_CODEC_LZ4F ? ((size_t)65536 << (2 * std::min(l, 3))) : ((size_t)32768 << l);
        t = std::max(t, frame_temp(frame_geo(B, n, F)).total);
    }
    return t;
}

// decode side: maxbpf descriptor slots per frame (blocks of 64 KiB / 32 KiB at the least)
static uint32_t frame_maxbpf(int codec, size_t F) {
    const size_t bmin = codec == LZH_CODEC_LZ4F ? 65536 : 32768;
    return (uint32_t)std::max<size_t>(1, (F + bmin - 1) / bmin);
}

size_t lzh_compress_temp_bytes(int codec, size_t n, size_t chunk_size) {
    size_t k = lzh_num_chunks(n, chunk_size);
    if (codec == LZH_CODEC_MEMCPY) return 256;
    if (is_frame(codec)) return frame_temp_worst(codec, n, chunk_size) + 256;
    size_t t = align_up(k * lzh_stage_stride(codec, chunk_size), 256) + 256;
    if (codec == LZH_CODEC_LZ4 && chunk_size <= kLz4SplitMax)     // sequence records of the parse kernel
        t += k * lzh_lz4_rec_stride(chunk_size) + align_up(k * 8, 256) + 256;
    if (codec == LZH_CODEC_SNAPPY && chunk_size <= kLz4SplitMax)
        t += k * lzh_snappy_rec_stride(chunk_size) + align_up(k * 4 * lzh_snappy_frags(chunk_size), 256) + 256;
    if (codec == LZH_CODEC_ZSTD) {   // per-frame scratch of the two zstd kernels (zstdc_hip.hip), worst level
        size_t fs = 0;
        for (int lv : {1, 2, -1, -2}) fs = std::max(fs, lzh_zstd_scratch_stride(chunk_size, lv));
        t += k * fs + 256;
    }
    return t;
}

size_t lzh_decompress_temp_bytes(int codec, size_t n, size_t chunk_size) {
    const size_t k = lzh_num_chunks(n, chunk_size);
    size_t t = align_up((k + 1) * sizeof(uint64_t), 256) + 256;
    if (is_frame(codec)) {   // block descriptors, block statuses, frame statuses
        const size_t nd = k * frame_maxbpf(codec, chunk_size);
        t += align_up(nd * 32, 256) + align_up(nd * 4, 256) + align_up(k * 4, 256) + 256;
    }
    if (codec == LZH_CODEC_ZSTD) t += lzh_zstd_decode_temp(n, chunk_size);   // the split decoder (decode_hip.hip)
    if (codec == LZH_CODEC_SNAPPY) t += lzh_snappy_split_temp(n, chunk_size); // fragment-parallel decode
    return t;
}

int lzh_compress_kernel_stage(int codec, int level, int stage_mask, const void* d_in, size_t n, size_t in_readable,
                              size_t chunk_size, void* d_stage, uint32_t* d_csizes, void* hip_stream) {
    hipStream_t s = (hipStream_t)hip_stream;
    if (!chunk_size || !d_stage || !d_csizes || (n && !d_in)) return LZH_EARG;
    const size_t k = lzh_num_chunks(n, chunk_size);
    if (k > 0xffffffffu || chunk_size > 0x7fff0000u) return LZH_EARG;
    const size_t stride = lzh_stage_stride(codec, chunk_size);
    Range range("lzh:compress_kernel");
    if (codec == LZH_CODEC_LZ4) {
        if (chunk_size <= kLz4SplitMax) {
            uint8_t* recs = (uint8_t*)d_stage + align_up(k * stride, 256) + 256;
            LZH_CHECK(lzh_launch_lz4_split((const uint8_t*)d_in, n, in_readable, chunk_size, level < 1 ? 1 : level,
                                           (uint8_t*)d_stage, stride, d_csizes, (uint32_t)k, recs, stage_mask, s));
        } else if (stage_mask & 1) {
            LZH_CHECK(lzh_launch_lz4_compress_v2((const uint8_t*)d_in, n, in_readable, chunk_size, level < 1 ? 1 : level,
                                                 (uint8_t*)d_stage, stride, d_csizes, (uint32_t)k, s));
        }
    } else if (codec == LZH_CODEC_SNAPPY) {
        if (chunk_size <= kLz4SplitMax) {
            uint8_t* recs = (uint8_t*)d_stage + align_up(k * stride, 256) + 256;
            LZH_CHECK(lzh_launch_snappy_split((const uint8_t*)d_in, n, in_readable, chunk_size, (uint8_t*)d_stage,
                                              stride, d_csizes, (uint32_t)k, recs, stage_mask, s));
        } else if (stage_mask & 1) {
            LZH_CHECK(lzh_launch_snappy_compress_v2((const uint8_t*)d_in, n, in_readable, chunk_size, (uint8_t*)d_stage,
                                                    stride, d_csizes, (uint32_t)k, s));
        }
    } else if (is_frame(codec)) {
        // (d_stage = the whole compression temp of a framed layout; d_csizes = frame sizes)
        if (!frame_level_ok(codec, level)) return LZH_EARG;
        const FrameGeo g = frame_geo(frame_block_bytes(codec, level), n, chunk_size);
        const FrameTemp t = frame_temp(g);
        uint8_t* base = (uint8_t*)d_stage;
        uint32_t* bcs = (uint32_t*)(base + t.bcs);
        const int acc = codec == LZH_CODEC_LZ4F ? std::max(1, (level >> 8) & 0xff) : 1;
        if (codec == LZH_CODEC_LZ4F && (level & LZH_LZ4F_LINKED)) {
            // linked blocks: one wave per frame walks its blocks in order (the records area holds the
            // per-frame table snapshots: 16 KiB per frame)
            if (stage_mask & 1)
                LZH_CHECK(lzh_launch_lz4f_linked((const uint8_t*)d_in, n, in_readable, g.F, g.bs, g.bpf, acc,
                                                 base + t.stage, t.stride, bcs, (uint32_t*)(base + t.recs),
                                                 (uint32_t)g.nframes, s));
        } else {
            LZH_CHECK(lzh_launch_lz4_split((const uint8_t*)d_in, n, in_readable, g.bs, acc, base + t.stage, t.stride, bcs,
                                           (uint32_t)g.nblocks, base + t.recs, stage_mask, s, g.F, g.bpf));
        }
        if (stage_mask & 2)
            LZH_CHECK(lzh_launch_frame_sizes(codec, level, n, g.F, g.bs, g.bpf, bcs, (uint32_t*)(base + t.rel), d_csizes,
                                             (uint32_t)g.nframes, s));
    } else if (codec == LZH_CODEC_ZSTD) {
        if (!lzh_zstd_level_ok(level, chunk_size)) return LZH_EARG;
        uint8_t* scratch = (uint8_t*)d_stage + align_up(k * stride, 256) + 256;
        if (stage_mask & 1)
            LZH_CHECK(lzh_launch_zstd_compress((const uint8_t*)d_in, n, in_readable, chunk_size, level,
                                               (uint8_t*)d_stage, stride, d_csizes, (uint32_t)k, scratch, s));
    } else {
        return LZH_EARG;
    }
    return LZH_OK;
}

int lzh_compress_kernel_only(int codec, int level, const void* d_in, size_t n, size_t in_readable,
                             size_t chunk_size, void* d_stage, uint32_t* d_csizes, void* hip_stream) {
    if (is_frame(codec)) return LZH_EARG;   // (framed layouts: lzh_compress_async)
    return lzh_compress_kernel_stage(codec, level, 3, d_in, n, in_readable, chunk_size, d_stage, d_csizes, hip_stream);
}

__global__ void lzh_fill_raw_sizes(uint32_t* cs, uint64_t k, uint64_t n, uint64_t chunk) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < k) cs[i] = (uint32_t)std::min<uint64_t>(chunk, n - i * chunk);
}

int lzh_compress_async(int codec, int level, const void* d_in, size_t n, size_t in_readable, size_t chunk_size,
                       void* d_packed, size_t packed_cap, uint32_t* d_csizes, uint64_t* d_offsets, void* d_temp,
                       size_t temp_bytes, void* hip_stream) {
    hipStream_t s = (hipStream_t)hip_stream;
    if (!chunk_size || !d_packed || !d_csizes || !d_offsets || (n && !d_in)) return LZH_EARG;
    if (in_readable < n) return LZH_EARG;
    const size_t k = lzh_num_chunks(n, chunk_size);
    if (codec == LZH_CODEC_MEMCPY) {
        if (packed_cap < n) return LZH_ESPACE;
        if (n == 0) return LZH_OK;
        hipLaunchKernelGGL(lzh_fill_raw_sizes, dim3((unsigned)((k + 255) / 256)), dim3(256), 0, s, d_csizes,
                           (uint64_t)k, (uint64_t)n, (uint64_t)chunk_size);
        LZH_CHECK(hipGetLastError());
        LZH_CHECK(lzh_launch_scan(d_csizes, k, d_offsets, nullptr, s));
        LZH_CHECK(lzh_launch_memcpy(d_in, d_packed, n, s));
        return LZH_OK;
    }
    if (temp_bytes < lzh_compress_temp_bytes(codec, n, chunk_size) || !d_temp) return LZH_ESPACE;
    if (packed_cap < lzh_max_packed_bytes(codec, n, chunk_size)) return LZH_ESPACE;
    if (is_frame(codec)) {   // blocks -> frame sizes -> frame offsets -> frames
        if (!frame_level_ok(codec, level)) return LZH_EARG;
        if (k > 0xffffffffu || chunk_size > 0x7fff0000u) return LZH_EARG;
        int rc = lzh_compress_kernel_stage(codec, level, 3, d_in, n, in_readable, chunk_size, d_temp, d_csizes, hip_stream);
        if (rc) return rc;
        const FrameGeo g = frame_geo(frame_block_bytes(codec, level), n, chunk_size);
        const FrameTemp t = frame_temp(g);
        const uint8_t* base = (const uint8_t*)d_temp;
        Range range("lzh:scan_pack");
        LZH_CHECK(lzh_launch_scan(d_csizes, k, d_offsets, nullptr, s));
        LZH_CHECK(lzh_launch_frame_pack(codec, level, (const uint8_t*)d_in, n, in_readable, g.F, g.bs, g.bpf,
                                        base + t.stage, t.stride, (const uint32_t*)(base + t.bcs),
                                        (const uint32_t*)(base + t.rel), d_csizes, d_offsets, (uint8_t*)d_packed,
                                        (uint32_t)g.nblocks, (uint32_t)g.nframes, s));
        return LZH_OK;
    }
    int rc = lzh_compress_kernel_only(codec, level, d_in, n, in_readable, chunk_size, d_temp, d_csizes, hip_stream);
    if (rc) return rc;
    return lzh_compress_finish_async(codec, d_in, n, in_readable, chunk_size, d_temp, d_csizes, d_packed, packed_cap,
                                     d_offsets, hip_stream);
}

int lzh_compress_finish_async(int codec, const void* d_in, size_t n, size_t in_readable, size_t chunk_size,
                              const void* d_stage, const uint32_t* d_csizes, void* d_packed, size_t packed_cap,
                              uint64_t* d_offsets, void* hip_stream) {
    hipStream_t s = (hipStream_t)hip_stream;
    if (!chunk_size || !d_stage || !d_csizes || !d_packed || !d_offsets) return LZH_EARG;
    if (codec != LZH_CODEC_LZ4 && codec != LZH_CODEC_SNAPPY && codec != LZH_CODEC_ZSTD) return LZH_EARG;
    // the sizes are only known on the device: the worst case must fit (no silent truncation)
    if (packed_cap < lzh_max_packed_bytes(codec, n, chunk_size)) return LZH_ESPACE;
    const size_t k = lzh_num_chunks(n, chunk_size);
    const size_t stride = lzh_stage_stride(codec, chunk_size);
    Range range("lzh:scan_pack");
    LZH_CHECK(lzh_launch_scan(d_csizes, k, d_offsets, nullptr, s));
    LZH_CHECK(lzh_launch_pack((const uint8_t*)d_in, n, in_readable, chunk_size, (const uint8_t*)d_stage, stride,
                              d_csizes, d_offsets, (uint8_t*)d_packed, packed_cap, (uint32_t)k, s));
    return LZH_OK;
}

int lzh_decompress_async(int codec, const void* d_packed, size_t packed_readable, const uint32_t* d_csizes,
                         const uint64_t* d_offsets, size_t n, size_t chunk_size, void* d_out, int32_t* d_status,
                         void* d_temp, size_t temp_bytes, void* hip_stream) {
    hipStream_t s = (hipStream_t)hip_stream;
    if (!chunk_size || !d_csizes || !d_status || (n && (!d_out || !d_packed))) return LZH_EARG;
    if (codec < 0 || codec > LZH_CODEC_NVLZ4) return LZH_EARG;
    if (codec == LZH_CODEC_ZSTD && chunk_size > (1u << 30)) return LZH_EARG;
    const size_t k = lzh_num_chunks(n, chunk_size);
    if (n == 0) return LZH_OK;
    Range range("lzh:decompress");
    const uint64_t* offs = d_offsets;
    const size_t scan_bytes = align_up((k + 1) * sizeof(uint64_t), 256);
    if (is_frame(codec) && (!d_temp || temp_bytes < lzh_decompress_temp_bytes(codec, n, chunk_size))) return LZH_ESPACE;
    if (!offs && (!d_temp || temp_bytes < scan_bytes + 256)) return LZH_ESPACE;
    // zstd: the split decoder's per-frame layout lives in temp after the offsets; without room for it
    // (or for chunks below lzh_zstd_split_min) every frame takes the one-wave decoder
    uint8_t* zt = nullptr;
    if (codec == LZH_CODEC_ZSTD && d_temp && temp_bytes >= lzh_decompress_temp_bytes(codec, n, chunk_size) &&
        lzh_zstd_decode_temp(n, chunk_size) > 0)
        zt = (uint8_t*)d_temp + scan_bytes;
    if (!offs) {
        LZH_CHECK(lzh_launch_scan(d_csizes, k, (uint64_t*)d_temp, nullptr, s));
        offs = (const uint64_t*)d_temp;
    }
    if (is_frame(codec)) {   // frame headers -> block descriptors -> blocks -> frame checks
        if (k > 0xffffffffu || chunk_size > 0x7fff0000u) return LZH_EARG;
        const uint32_t mb = frame_maxbpf(codec, chunk_size);
        const size_t nd = k * mb;
        uint8_t* t = (uint8_t*)d_temp + align_up((k + 1) * sizeof(uint64_t), 256);
        void* desc = t;
        int32_t* bstat = (int32_t*)(t + align_up(nd * 32, 256));
        int32_t* fstat = (int32_t*)(t + align_up(nd * 32, 256) + align_up(nd * 4, 256));
        if (nd > 0xffffffffu) return LZH_EARG;
        LZH_CHECK(lzh_launch_frame_parse(codec, (const uint8_t*)d_packed, packed_readable, offs, d_csizes, n, chunk_size,
                                         mb, desc, fstat, (uint32_t)k, s));
        LZH_CHECK(lzh_launch_decompress(LZH_CODEC_LZ4, (const uint8_t*)d_packed, packed_readable, nullptr, nullptr, n,
                                        chunk_size, (uint8_t*)d_out, bstat, (uint32_t)nd, s, desc));
        LZH_CHECK(lzh_launch_frame_finish(codec, (const uint8_t*)d_packed, offs, d_csizes, n, chunk_size, mb, desc,
                                          bstat, fstat, (const uint8_t*)d_out, d_status, (uint32_t)k, s));
        return LZH_OK;
    }
    // snappy chunks of several 64 KiB fragments decode a fragment per wave when temp has room for the split
    // (else, or for chunks of one fragment, whole)
    const size_t sst = codec == LZH_CODEC_SNAPPY ? lzh_snappy_split_temp(n, chunk_size) : 0;
    if (codec == LZH_CODEC_ZSTD)
        LZH_CHECK(lzh_launch_zstd_decompress((const uint8_t*)d_packed, packed_readable, offs, d_csizes, n, chunk_size,
                                             (uint8_t*)d_out, d_status, (uint32_t)k, zt, s));
    else if (sst && d_temp && temp_bytes >= scan_bytes + sst)
        LZH_CHECK(lzh_launch_snappy_split_decompress((const uint8_t*)d_packed, packed_readable, offs, d_csizes, n,
                                                     chunk_size, (uint8_t*)d_out, d_status, (uint32_t)k,
                                                     (uint8_t*)d_temp + scan_bytes, s));
    else
        LZH_CHECK(lzh_launch_decompress(codec, (const uint8_t*)d_packed, packed_readable, offs, d_csizes, n,
                                        chunk_size, (uint8_t*)d_out, d_status, (uint32_t)k, s));
    return LZH_OK;
}

}  // extern "C"

// ======================================================================= host layer

namespace {

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = align_up(bytes + 4096, 1 << 20);
        if (hipMalloc(&p, want) != hipSuccess) { p = nullptr; (void)hipGetLastError(); return -1; }
        cap = want;
        return 0;
    }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
};

// the calling thread's current device is restored on every exit path of a row function
// (lzbench's process -- or a torch rank -- keeps allocating on the device it selected)
struct DeviceGuard {
    int prev = -1;
    DeviceGuard() { if (hipGetDevice(&prev) != hipSuccess) prev = -1; }
    ~DeviceGuard() { if (prev >= 0) (void)hipSetDevice(prev); }
};

struct Dev {
    int id = 0;
    hipStream_t s = nullptr;      // kernels (even sub-batches)
    hipStream_t s2 = nullptr;     // kernels (odd sub-batches: overlaps the tail of the previous grid)
    hipStream_t sin = nullptr;    // host -> device copies
    hipStream_t sout = nullptr;   // device -> host copies
    DevBuf in, packed, temp, temp2, csizes, offsets, status;
    uint32_t* h_cs = nullptr;     // pinned: chunk sizes / statuses read back per sub-batch
    size_t h_cap = 0;
    int ensure_host(size_t n) {
        if (n <= h_cap) return 0;
        if (h_cs) (void)hipHostFree(h_cs);
        h_cs = nullptr;
        h_cap = 0;
        if (hipHostMalloc((void**)&h_cs, std::max<size_t>(n, 1024) * 4, hipHostMallocDefault) != hipSuccess) return -1;
        h_cap = std::max<size_t>(n, 1024);
        return 0;
    }
};

struct HostReg { void* p; size_t n; };

struct LzhCtx {
    uint32_t magic = 0x4c5a4858;  // "LZHX"
    int codec = 0;
    size_t chunk_size = 0;
    std::vector<Dev> devs;        // logical shards (may outnumber the physical devices)
    std::vector<HostReg> regs;    // host ranges page-locked by this row (lzbench reuses its buffers)
};

LzhCtx* ctx_of(char* wm) {
    LzhCtx* c = (LzhCtx*)wm;
    return (c && c->magic == 0x4c5a4858) ? c : nullptr;
}

// page-lock [p, p+n) once per row so the copies run at PCIe rate and asynchronously (the
// reference driver hands over pageable malloc'd buffers, lzbench.cpp:256-263); a range that
// cannot be registered is simply copied from pageable memory
void ensure_pinned(LzhCtx* c, const void* p, size_t n) {
    if (!p || n < (1u << 20)) return;
    const uintptr_t a0 = (uintptr_t)p & ~(uintptr_t)4095, a1 = ((uintptr_t)p + n + 4095) & ~(uintptr_t)4095;
    for (const HostReg& r : c->regs)
        if ((uintptr_t)r.p <= a0 && a1 <= (uintptr_t)r.p + r.n) return;
    if (hipHostRegister((void*)a0, a1 - a0, hipHostRegisterPortable) == hipSuccess) c->regs.push_back({(void*)a0, a1 - a0});
    else (void)hipGetLastError();
}

void ctx_free(LzhCtx* c) {
    DeviceGuard guard;
    for (Dev& d : c->devs) {
        (void)hipSetDevice(d.id);
        d.in.release(); d.packed.release(); d.temp.release(); d.temp2.release(); d.csizes.release(); d.offsets.release();
        d.status.release();
        if (d.h_cs) (void)hipHostFree(d.h_cs);
        if (d.s) (void)hipStreamDestroy(d.s);
        if (d.s2) (void)hipStreamDestroy(d.s2);
        if (d.sin) (void)hipStreamDestroy(d.sin);
        if (d.sout) (void)hipStreamDestroy(d.sout);
    }
    for (const HostReg& r : c->regs) (void)hipHostUnregister(r.p);
    c->magic = 0;
    delete c;
}

// ngpus logical shards (lzbench's additional_param of the row) starting at the caller's current
// device; shard g runs on device (current + g) mod count, so ngpus larger than the visible device
// count is legal (several shards share a device on their own streams; results are identical)
char* ctx_new(int codec, size_t chunk_size, size_t ngpus) {
    DeviceGuard guard;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        fprintf(stderr, "lzbench_hip: no HIP device available\n");
        return nullptr;
    }
    if (ngpus == 0) ngpus = 1;
    if (ngpus > 64) ngpus = 64;
    const int base = guard.prev >= 0 ? guard.prev : 0;
    LzhCtx* c = new LzhCtx();
    c->codec = codec;
    c->chunk_size = chunk_size;
    c->devs.resize(ngpus);
    for (size_t g = 0; g < ngpus; g++) {
        Dev& d = c->devs[g];
        d.id = (int)((base + g) % (size_t)count);
        if (hipSetDevice(d.id) != hipSuccess || hipStreamCreateWithFlags(&d.s, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&d.s2, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&d.sin, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&d.sout, hipStreamNonBlocking) != hipSuccess) {
            fprintf(stderr, "lzbench_hip: cannot open device %d\n", d.id);
            ctx_free(c);
            return nullptr;
        }
    }
    return (char*)c;
}

// chunks per pipelined sub-batch: ~128 MiB of input and at least 1 024 chunks (a full grid round
// of the widest-LDS kernel); consecutive sub-batches of a device alternate between two kernel
// streams so a grid's tail overlaps the next grid.  With several shards the sub-batch shrinks
// until every shard owns at least two.
size_t sub_batch_chunks(size_t chunk, size_t k, size_t G) {
    size_t sbk = std::max<size_t>(1024, ((size_t)128 << 20) / std::max<size_t>(chunk, 1));
    if (G > 1) sbk = std::min(sbk, std::max<size_t>(1, (k + 2 * G - 1) / (2 * G)));
    return sbk;
}

struct Events {
    std::vector<hipEvent_t> ev;
    hipEvent_t get(size_t i) {
        while (ev.size() <= i) {
            hipEvent_t e = nullptr;
            if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
            ev.push_back(e);
        }
        return ev[i];
    }
    ~Events() { for (hipEvent_t e : ev) (void)hipEventDestroy(e); }
};

// Sharding plan of one run (k chunks of `chunk` bytes covering n bytes): sub-batch j = chunks
// [j*sbk, min(k, (j+1)*sbk)) goes to shard j mod G as that shard's local slot j / G.  Every
// shard owns a contiguous set of index ranges, and the sub-batches finish roughly in index order
// across all shards, so the host gather (which must place sub-batch j after everything before
// it, lzbench.cpp:266-298 packing) can copy each one out as soon as its sizes land instead of
// waiting for whole shards in shard order.
struct Plan {
    size_t k, sbk, nsb, G;
    size_t chunk, n;
    size_t c_begin(size_t j) const { return j * sbk; }
    size_t c_count(size_t j) const { return std::min(sbk, k - j * sbk); }
    size_t b_begin(size_t j) const { return j * sbk * chunk; }
    size_t b_count(size_t j) const { return std::min(n, (j * sbk + c_count(j)) * chunk) - b_begin(j); }
    size_t shard(size_t j) const { return j % G; }
    size_t slot(size_t j) const { return j / G; }
    size_t slots(size_t g) const { return nsb > g ? (nsb - g + G - 1) / G : 0; }
};

// Host gather bookkeeping (pure host code, tested on the CPU through lzh_debug_gather_order):
// sub-batches finish in any order across the shards; sub-batch j's packed bytes go to the
// output at the sum of the packed sizes before it (lzbench.cpp:266-298), so j is placed as soon
// as its own sizes and every earlier sub-batch's are known -- the earliest moment its offset
// exists -- and the copies leave in chunk order.
struct GatherOrder {
    std::vector<uint8_t> done;
    std::vector<size_t> tot;
    size_t next = 0, base = 0;
    explicit GatherOrder(size_t n) : done(n, 0), tot(n, 0) {}
    bool finished() const { return next == done.size(); }
    // j's sizes are known (packed total t): place(j', offset) for every sub-batch that became placeable
    template <class F>
    int complete(size_t j, size_t t, F&& place) {
        done[j] = 1;
        tot[j] = t;
        while (next < done.size() && done[next]) {
            const int rc = place(next, base);
            if (rc) return rc;
            base += tot[next];
            next++;
        }
        return 0;
    }
};

// (a chunk size above the input is one chunk of the input's size: buffers are sized from the bytes
// present, not from lzbench's 1.79 GB default chunk)
size_t row_chunk(size_t n, size_t chunk) { return std::max<size_t>(std::min(chunk, n), 1); }

Plan make_plan(size_t ndev, size_t n, size_t chunk) {
    Plan p;
    p.n = n;
    p.chunk = chunk;
    p.k = lzh_num_chunks(n, chunk);
    p.G = std::max<size_t>(1, std::min(ndev, p.k));
    p.sbk = sub_batch_chunks(chunk, p.k, p.G);
    p.nsb = (p.k + p.sbk - 1) / p.sbk;
    p.G = std::min(p.G, p.nsb);
    return p;
}

// process one run: chunks [0, k) of uniform size `chunk` (last ragged) covering n bytes of
// host input; results appended at out (capacity outcap). Returns packed bytes, 0 when the
// packed output does not fit outcap, < 0 on error.  Per shard, sub-batches are pipelined over
// three streams (host->device copy | compress + scan + pack | device->host copy).
int64_t run_compress(LzhCtx* c, int level, const uint8_t* in, size_t n, size_t chunk, uint8_t* out, size_t outcap,
                     size_t* compr_sizes) {
    DeviceGuard guard;
    Range range("lzh:row_compress");
    chunk = row_chunk(n, chunk);
    const Plan P = make_plan(c->devs.size(), n, chunk);
    const size_t sb_in = std::min(n, P.sbk * chunk);                   // largest sub-batch input
    const size_t sb_packed = align_up(lzh_max_packed_bytes(c->codec, sb_in, chunk) + 64, 256);
    const size_t sb_temp = lzh_compress_temp_bytes(c->codec, sb_in, chunk);
    ensure_pinned(c, in, n);
    ensure_pinned(c, out, outcap);
    for (size_t g = 0; g < P.G; g++) {
        Dev& d = c->devs[g];
        const size_t m = P.slots(g);
        if (hipSetDevice(d.id) != hipSuccess) return LZH_EHIP;
        if (d.in.ensure(m * sb_in + 64) || d.packed.ensure(m * sb_packed) || d.temp.ensure(sb_temp) ||
            (m > 1 && d.temp2.ensure(sb_temp)) || d.csizes.ensure(m * P.sbk * 4 + 64) ||
            d.offsets.ensure(m * (P.sbk + 1) * 8 + 64) || d.ensure_host(m * P.sbk))
            return LZH_ESPACE;
    }
    Events evin, evk;
    for (size_t j = 0; j < P.nsb; j++) {     // issue every sub-batch, round-robin over the shards
        Dev& d = c->devs[P.shard(j)];
        const size_t l = P.slot(j), ck = P.c_count(j), rn = P.b_count(j);
        if (hipSetDevice(d.id) != hipSuccess) return LZH_EHIP;
        hipEvent_t e_in = evin.get(j), e_k = evk.get(j);
        if (!e_in || !e_k) return LZH_EHIP;
        uint8_t* din = (uint8_t*)d.in.p + l * sb_in;
        LZH_CHECK(hipMemcpyAsync(din, in + P.b_begin(j), rn, hipMemcpyHostToDevice, d.sin));
        hipStream_t ks = (l & 1) ? d.s2 : d.s;
        DevBuf& tb = (l & 1) ? d.temp2 : d.temp;
        LZH_CHECK(hipEventRecord(e_in, d.sin));
        LZH_CHECK(hipStreamWaitEvent(ks, e_in, 0));
        uint32_t* dcs = (uint32_t*)d.csizes.p + l * P.sbk;
        int rc = lzh_compress_async(c->codec, level, din, rn, rn + 64, chunk, (uint8_t*)d.packed.p + l * sb_packed,
                                    sb_packed, dcs, (uint64_t*)d.offsets.p + l * (P.sbk + 1), tb.p, tb.cap, ks);
        if (rc) return rc;
        LZH_CHECK(hipMemcpyAsync(d.h_cs + l * P.sbk, dcs, ck * 4, hipMemcpyDeviceToHost, ks));
        LZH_CHECK(hipEventRecord(e_k, ks));
    }
    // host-side gather: block on the next sub-batch in chunk order (its offset needs every earlier
    // one), then take any later sub-batch that has already finished on another shard without
    // waiting; copies leave as soon as their chunk-order offset is known
    bool fits = true;
    GatherOrder go(P.nsb);
    auto place = [&](size_t j, size_t base) -> int {
        Dev& d = c->devs[P.shard(j)];
        const size_t l = P.slot(j), tot = go.tot[j];
        if (!fits || base + tot > outcap) { fits = false; return 0; }   // lzbench: cannot store
        if (hipSetDevice(d.id) != hipSuccess) return LZH_EHIP;
        LZH_CHECK(hipStreamWaitEvent(d.sout, evk.get(j), 0));
        LZH_CHECK(hipMemcpyAsync(out + base, (uint8_t*)d.packed.p + l * sb_packed, tot, hipMemcpyDeviceToHost, d.sout));
        return 0;
    };
    auto take = [&](size_t j) -> int {   // j's kernels and size copy are done: record its sizes
        Dev& d = c->devs[P.shard(j)];
        const size_t l = P.slot(j), ck = P.c_count(j), c0 = P.c_begin(j);
        size_t tot = 0;
        const uint32_t* hs = d.h_cs + l * P.sbk;
        for (size_t i = 0; i < ck; i++) { compr_sizes[c0 + i] = hs[i]; tot += hs[i]; }
        return go.complete(j, tot, place);
    };
    while (!go.finished()) {
        const size_t j0 = go.next;
        hipError_t q = hipEventSynchronize(evk.get(j0));
        if (q != hipSuccess) {
            fprintf(stderr, "lzbench_hip: sub-batch %zu failed: %s\n", j0, hipGetErrorString(q));
            return LZH_EHIP;
        }
        if (const int rc = take(j0)) return rc;
        for (size_t j = go.next; j < P.nsb; j++) {
            if (go.done[j]) continue;
            q = hipEventQuery(evk.get(j));
            if (q == hipErrorNotReady) continue;
            if (q != hipSuccess) {
                fprintf(stderr, "lzbench_hip: sub-batch %zu failed: %s\n", j, hipGetErrorString(q));
                return LZH_EHIP;
            }
            if (const int rc = take(j)) return rc;
        }
    }
    const size_t base = go.base;
    for (size_t g = 0; g < P.G; g++) {
        if (hipSetDevice(c->devs[g].id) != hipSuccess || hipStreamSynchronize(c->devs[g].sout) != hipSuccess ||
            hipStreamSynchronize(c->devs[g].s) != hipSuccess || hipStreamSynchronize(c->devs[g].s2) != hipSuccess)
            return LZH_EHIP;
    }
    return fits ? (int64_t)base : 0;
}

// Inverse of run_compress over the same plan.  Returns the decoded byte count (== n) or < 0:
// a chunk whose decoder reports anything but its own size is malformed (LZH_ECORRUPT), which
// keeps lzbench's length check (lzbench.cpp:433-437) honest for short decodes.
int64_t run_decompress(LzhCtx* c, const uint8_t* in, const size_t* compr_sizes, size_t n, size_t chunk, uint8_t* out) {
    DeviceGuard guard;
    Range range("lzh:row_decompress");
    chunk = row_chunk(n, chunk);
    const Plan P = make_plan(c->devs.size(), n, chunk);
    const size_t k = P.k;
    std::vector<size_t> coff(k + 1, 0);
    for (size_t i = 0; i < k; i++) coff[i + 1] = coff[i] + compr_sizes[i];
    size_t sb_cin = 0;                        // largest compressed sub-batch
    for (size_t j = 0; j < P.nsb; j++)
        sb_cin = std::max(sb_cin, coff[P.c_begin(j) + P.c_count(j)] - coff[P.c_begin(j)]);
    sb_cin = align_up(sb_cin + 64, 256);
    const size_t sb_out = std::min(n, P.sbk * chunk);
    const size_t sb_temp = lzh_decompress_temp_bytes(c->codec, sb_out, chunk);
    ensure_pinned(c, in, coff[k]);
    ensure_pinned(c, out, n);
    for (size_t g = 0; g < P.G; g++) {
        Dev& d = c->devs[g];
        const size_t m = P.slots(g);
        if (hipSetDevice(d.id) != hipSuccess) return LZH_EHIP;
        if (d.in.ensure(m * sb_cin) || d.packed.ensure(m * sb_out + 64) || d.csizes.ensure(m * P.sbk * 4 + 64) ||
            d.status.ensure(m * P.sbk * 4 + 64) || d.temp.ensure(sb_temp) || d.temp2.ensure(sb_temp) ||
            d.ensure_host(2 * m * P.sbk))
            return LZH_ESPACE;
    }
    Events evin, evk;
    for (size_t j = 0; j < P.nsb; j++) {
        Dev& d = c->devs[P.shard(j)];
        const size_t l = P.slot(j), m = P.slots(P.shard(j)), ck = P.c_count(j), c0 = P.c_begin(j);
        const size_t rn = P.b_count(j), po = coff[c0], pn = coff[c0 + ck] - po;
        if (hipSetDevice(d.id) != hipSuccess) return LZH_EHIP;
        hipEvent_t e_in = evin.get(j), e_k = evk.get(j);
        if (!e_in || !e_k) return LZH_EHIP;
        uint32_t* h_in = d.h_cs + l * P.sbk;                  // sizes in
        for (size_t i = 0; i < ck; i++) h_in[i] = (uint32_t)compr_sizes[c0 + i];
        uint8_t* din = (uint8_t*)d.in.p + l * sb_cin;
        uint32_t* dcs = (uint32_t*)d.csizes.p + l * P.sbk;
        int32_t* dst = (int32_t*)d.status.p + l * P.sbk;
        uint8_t* dout = (uint8_t*)d.packed.p + l * sb_out;
        LZH_CHECK(hipMemcpyAsync(din, in + po, pn, hipMemcpyHostToDevice, d.sin));
        LZH_CHECK(hipMemcpyAsync(dcs, h_in, ck * 4, hipMemcpyHostToDevice, d.sin));
        LZH_CHECK(hipEventRecord(e_in, d.sin));
        hipStream_t ks = (l & 1) ? d.s2 : d.s;
        DevBuf& tb = (l & 1) ? d.temp2 : d.temp;
        LZH_CHECK(hipStreamWaitEvent(ks, e_in, 0));
        int rc = lzh_decompress_async(c->codec, din, pn + 64, dcs, nullptr, rn, chunk, dout, dst, tb.p, tb.cap, ks);
        if (rc) return rc;
        LZH_CHECK(hipEventRecord(e_k, ks));
        LZH_CHECK(hipStreamWaitEvent(d.sout, e_k, 0));
        int32_t* h_st = (int32_t*)d.h_cs + m * P.sbk + l * P.sbk;   // statuses out
        LZH_CHECK(hipMemcpyAsync(h_st, dst, ck * 4, hipMemcpyDeviceToHost, d.sout));
        LZH_CHECK(hipMemcpyAsync(out + P.b_begin(j), dout, rn, hipMemcpyDeviceToHost, d.sout));
    }
    for (size_t g = 0; g < P.G; g++) {
        Dev& d = c->devs[g];
        if (hipSetDevice(d.id) != hipSuccess || hipStreamSynchronize(d.sout) != hipSuccess ||
            hipStreamSynchronize(d.s) != hipSuccess || hipStreamSynchronize(d.s2) != hipSuccess)
            return LZH_EHIP;
    }
    int64_t sum = 0;
    bool bad = false;
    for (size_t j = 0; j < P.nsb; j++) {
        const Dev& d = c->devs[P.shard(j)];
        const size_t l = P.slot(j), m = P.slots(P.shard(j)), ck = P.c_count(j), c0 = P.c_begin(j);
        const int32_t* h_st = (const int32_t*)d.h_cs + m * P.sbk + l * P.sbk;
        for (size_t i = 0; i < ck; i++) {
            const int64_t part = (int64_t)std::min(chunk, n - (c0 + i) * chunk);
            if (h_st[i] != part) bad = true;
            sum += h_st[i];
        }
    }
    return bad ? LZH_ECORRUPT : sum;
}

}  // namespace

// debug (CPU): the gather's placement order for sub-batches completing in `order` with packed
// sizes `sizes`: placed[i] = (sub-batch, offset, index into `order` of the completion that placed it)
extern "C" int lzh_debug_gather_order(size_t nsb, const uint64_t* order, const uint64_t* sizes, uint64_t* placed) {
    GatherOrder go(nsb);
    size_t np = 0, at = 0;
    for (size_t i = 0; i < nsb; i++) {
        at = i;
        go.complete((size_t)order[i], (size_t)sizes[order[i]], [&](size_t j, size_t base) {
            placed[3 * np] = j;
            placed[3 * np + 1] = base;
            placed[3 * np + 2] = at;
            np++;
            return 0;
        });
    }
    return (int)np;
}

extern "C" int lzh_debug_plan(size_t ngpus, size_t n, size_t chunk_size, int codec, uint64_t* out, int nout) {
    if (!out || nout <= 0 || chunk_size == 0) return 0;
    chunk_size = row_chunk(n, chunk_size);
    const Plan P = make_plan(std::max<size_t>(std::min<size_t>(ngpus, 64), 1), n, chunk_size);
    const size_t sb_in = std::min(n, P.sbk * chunk_size);
    std::vector<uint64_t> v = {P.k, P.sbk, P.nsb, P.G, sb_in,
                               align_up(lzh_max_packed_bytes(codec, sb_in, chunk_size) + 64, 256),
                               lzh_compress_temp_bytes(codec, sb_in, chunk_size)};
    for (size_t g = 0; g < P.G; g++) v.push_back(P.slots(g));
    const int m = std::min<int>(nout, (int)v.size());
    for (int i = 0; i < m; i++) out[i] = v[i];
    return m;
}

namespace {

int64_t one_chunk_compress(int codec_expect, char* in, size_t insize, char* out, size_t outsize, size_t level, char* wm) {
    LzhCtx* c = ctx_of(wm);
    if (!c || c->codec != codec_expect) return 0;
    size_t cs = 0;
    const size_t chunk = std::max<size_t>(insize, 1);
    int64_t r = run_compress(c, (int)level, (const uint8_t*)in, insize, chunk, (uint8_t*)out, outsize, &cs);
    return r <= 0 ? 0 : (int64_t)cs;
}

int64_t one_chunk_decompress(int codec_expect, char* in, size_t insize, char* out, size_t outsize, char* wm) {
    LzhCtx* c = ctx_of(wm);
    if (!c || c->codec != codec_expect) return 0;
    size_t cs = insize;
    const size_t chunk = std::max<size_t>(outsize, 1);
    return run_decompress(c, (const uint8_t*)in, &cs, outsize, chunk, (uint8_t*)out);
}

}  // namespace

extern "C" {

char* lzbench_hip_lz4_init(size_t chunk_size, size_t level, size_t ngpus) { (void)level; return ctx_new(LZH_CODEC_LZ4, chunk_size, ngpus); }
char* lzbench_hip_snappy_init(size_t chunk_size, size_t level, size_t ngpus) { (void)level; return ctx_new(LZH_CODEC_SNAPPY, chunk_size, ngpus); }
char* lzbench_hip_memcpy_init(size_t chunk_size, size_t level, size_t ngpus) { (void)level; return ctx_new(LZH_CODEC_MEMCPY, chunk_size, ngpus); }
char* lzbench_hip_zstd_init(size_t chunk_size, size_t level, size_t ngpus) { (void)level; return ctx_new(LZH_CODEC_ZSTD, chunk_size, ngpus); }
char* lzbench_hip_lz4frame_init(size_t chunk_size, size_t level, size_t ngpus) { (void)level; return ctx_new(LZH_CODEC_LZ4F, chunk_size, ngpus); }
char* lzbench_hip_nvcomp_lz4_init(size_t chunk_size, size_t level, size_t ngpus) { (void)level; return ctx_new(LZH_CODEC_NVLZ4, chunk_size, ngpus); }

void lzbench_hip_deinit(char* wm) {
    LzhCtx* c = ctx_of(wm);
    if (c) ctx_free(c);
}

int64_t lzbench_hip_lz4_compress(char* in, size_t insize, char* out, size_t outsize, size_t, size_t, char* wm) {
    return one_chunk_compress(LZH_CODEC_LZ4, in, insize, out, outsize, 1, wm);
}
int64_t lzbench_hip_lz4fast_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t, char* wm) {
    return one_chunk_compress(LZH_CODEC_LZ4, in, insize, out, outsize, level, wm);
}
int64_t lzbench_hip_lz4_decompress(char* in, size_t insize, char* out, size_t outsize, size_t, size_t, char* wm) {
    return one_chunk_decompress(LZH_CODEC_LZ4, in, insize, out, outsize, wm);
}
int64_t lzbench_hip_snappy_compress(char* in, size_t insize, char* out, size_t outsize, size_t, size_t, char* wm) {
    return one_chunk_compress(LZH_CODEC_SNAPPY, in, insize, out, outsize, 0, wm);
}
int64_t lzbench_hip_snappy_decompress(char* in, size_t insize, char* out, size_t outsize, size_t, size_t, char* wm) {
    return one_chunk_decompress(LZH_CODEC_SNAPPY, in, insize, out, outsize, wm);
}
int64_t lzbench_hip_zstd_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t, char* wm) {
    return one_chunk_compress(LZH_CODEC_ZSTD, in, insize, out, outsize, level, wm);
}
int64_t lzbench_hip_zstd_decompress(char* in, size_t insize, char* out, size_t outsize, size_t, size_t, char* wm) {
    return one_chunk_decompress(LZH_CODEC_ZSTD, in, insize, out, outsize, wm);
}
int64_t lzbench_hip_lz4frame_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t, char* wm) {
    return one_chunk_compress(LZH_CODEC_LZ4F, in, insize, out, outsize, level, wm);
}
int64_t lzbench_hip_lz4frame_decompress(char* in, size_t insize, char* out, size_t outsize, size_t, size_t, char* wm) {
    return one_chunk_decompress(LZH_CODEC_LZ4F, in, insize, out, outsize, wm);
}
int64_t lzbench_hip_nvcomp_lz4_compress(char* in, size_t insize, char* out, size_t outsize, size_t level, size_t, char* wm) {
    return one_chunk_compress(LZH_CODEC_NVLZ4, in, insize, out, outsize, level, wm);
}
int64_t lzbench_hip_nvcomp_lz4_decompress(char* in, size_t insize, char* out, size_t outsize, size_t, size_t, char* wm) {
    return one_chunk_decompress(LZH_CODEC_NVLZ4, in, insize, out, outsize, wm);
}
int64_t lzbench_hip_memcpy(char* in, size_t insize, char* out, size_t outsize, size_t, size_t, char* wm) {
    LzhCtx* c = ctx_of(wm);
    if (!c || outsize < insize) return 0;
    DeviceGuard guard;
    Dev& d = c->devs[0];
    if (hipSetDevice(d.id) != hipSuccess || d.in.ensure(insize + 64)) return 0;
    ensure_pinned(c, in, insize);
    ensure_pinned(c, out, outsize);
    if (hipMemcpyAsync(d.in.p, in, insize, hipMemcpyHostToDevice, d.s) != hipSuccess ||
        hipMemcpyAsync(out, d.in.p, insize, hipMemcpyDeviceToHost, d.s) != hipSuccess ||
        hipStreamSynchronize(d.s) != hipSuccess)
        return 0;
    return (int64_t)insize;
}

int64_t lzbench_hip_compress_batch(const char* in, const size_t* chunk_sizes, int nchunks, char* out, size_t outcap,
                                   size_t* compr_sizes, size_t level, size_t, char* wm) {
    LzhCtx* c = ctx_of(wm);
    if (!c || nchunks < 0) return 0;
    // runs of uniform chunking: a run ends after a chunk shorter than the first of the run
    int64_t total = 0;
    size_t ipos = 0;
    int i = 0;
    while (i < nchunks) {
        const size_t chunk = chunk_sizes[i];
        int j = i;
        size_t n = 0;
        while (j < nchunks && chunk_sizes[j] <= chunk) {
            n += chunk_sizes[j];
            if (chunk_sizes[j++] < chunk) break;
        }
        int64_t r = run_compress(c, (int)level, (const uint8_t*)in + ipos, n, std::max<size_t>(chunk, 1),
                                 (uint8_t*)out + total, outcap - (size_t)total, compr_sizes + i);
        if (r <= 0 && n > 0) return r;
        total += r;
        ipos += n;
        i = j;
    }
    return total;
}

int64_t lzbench_hip_decompress_batch(const char* in, const size_t* compr_sizes, const size_t* chunk_sizes, int nchunks,
                                     char* out, size_t outcap, size_t, size_t, char* wm) {
    LzhCtx* c = ctx_of(wm);
    if (!c || nchunks < 0) return 0;
    int64_t total = 0;
    size_t ipos = 0;
    int i = 0;
    while (i < nchunks) {
        const size_t chunk = chunk_sizes[i];
        int j = i;
        size_t n = 0, cn = 0;
        while (j < nchunks && chunk_sizes[j] <= chunk) {
            n += chunk_sizes[j];
            cn += compr_sizes[j];
            if (chunk_sizes[j++] < chunk) break;
        }
        if ((size_t)total + n > outcap) return 0;
        int64_t r = run_decompress(c, (const uint8_t*)in + ipos, compr_sizes + i, n, std::max<size_t>(chunk, 1),
                                   (uint8_t*)out + total);
        if (r < 0) return r;
        total += (int64_t)n;
        ipos += cn;
        i = j;
    }
    return total;
}

}  // extern "C"
