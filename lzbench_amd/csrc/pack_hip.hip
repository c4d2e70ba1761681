// lzbench_amd/csrc/pack_hip.hip -- device side of lzbench's packing convention
// (reference _lzbench/lzbench.cpp:266-298): per-chunk compressed sizes are scanned into
// output offsets, a chunk whose compressed size equals its raw size is stored raw, and the
// chunks are concatenated in chunk order.  Also the device memcpy used by the
// hipMemcpy-style plumbing row.
#include "common.h"

// exclusive scan of csizes[0..nchunks) -> offsets[0..nchunks], offsets[nchunks] = total
extern "C" __global__ void __launch_bounds__(1024)
lzh_scan_kernel(const uint32_t* csizes, uint64_t nchunks, uint64_t* offsets, uint64_t* total_out) {
    __shared__ uint64_t part[1024];
    const int t = threadIdx.x;
    const uint64_t per = (nchunks + 1023) / 1024;
    const uint64_t b = per * t, e = min<uint64_t>(b + per, nchunks);
    uint64_t s = 0;
    for (uint64_t i = b; i < e; i++) s += csizes[i];
    part[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {   // Hillis-Steele inclusive scan of the partials
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = t ? part[t - 1] : 0;
    for (uint64_t i = b; i < e; i++) { offsets[i] = run; run += csizes[i]; }
    if (t == 1023) {
        offsets[nchunks] = part[1023];
        if (total_out) *total_out = part[1023];
    }
}

// one workgroup per chunk: packed[offsets[c] ..] = raw input or staged stream
extern "C" __global__ void __launch_bounds__(256)
lzh_pack_kernel(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                const uint8_t* stage, uint64_t stride, const uint32_t* csizes, const uint64_t* offsets,
                uint8_t* packed, uint64_t packed_cap) {
    const uint64_t c = blockIdx.x;
    const uint64_t ioff = c * chunk_size;
    if (ioff >= n_total) return;
    const uint32_t part = (uint32_t)min(chunk_size, n_total - ioff);
    const uint32_t cs = csizes[c];
    const uint64_t doff = offsets[c];
    if (doff + cs > packed_cap) return;   // caller sized packed from offsets[nchunks]
    const bool raw = cs == part;
    const uint8_t* sp = raw ? in + ioff : stage + c * stride;
    const uint64_t sread = raw ? min<uint64_t>(in_readable - ioff, (uint64_t)part + 8) : stride;
    Bytes src, dst;
    src.init(sp, sread);
    dst.init(packed + doff, cs);
    // 16 bytes per thread and step: destination-aligned 16-byte stores, each from five aligned source
    // dwords shifted by v_alignbyte; bytewise head (to the destination's 16-byte boundary) and tail
    const int t = threadIdx.x, nt = blockDim.x, n = (int)cs;
    const int head = min(n, (int)((16u - ((uint32_t)(uint64_t)(packed + doff) & 15u)) & 15u));
    if (t < head) dst.st8(t, src.b(t));
    const int nb = (n - head) >> 4;
    for (int k = t; k < nb; k += nt) {
        const int p = head + 16 * k;                       // source / destination position
        const int Y = p + src.sh, Y0 = Y & ~3;
        const uint32_t sft = (uint32_t)Y & 3u;
        const uint32_t d0 = ld_b32(src.r, Y0), d1 = ld_b32(src.r, Y0 + 4), d2 = ld_b32(src.r, Y0 + 8),
                       d3 = ld_b32(src.r, Y0 + 12), d4 = ld_b32(src.r, Y0 + 16);
        const u32x4 v = {__builtin_amdgcn_alignbyte(d1, d0, sft), __builtin_amdgcn_alignbyte(d2, d1, sft),
                         __builtin_amdgcn_alignbyte(d3, d2, sft), __builtin_amdgcn_alignbyte(d4, d3, sft)};
        __builtin_amdgcn_raw_buffer_store_b128(v, dst.r, p + dst.sh, 0, 0);
    }
    const int t0 = head + 16 * nb;
    if (t < n - t0) dst.st8(t0 + t, src.b(t0 + t));
}

// plain device copy, 16 B per lane (plumbing row: device memcpy of the whole input)
extern "C" __global__ void __launch_bounds__(256)
lzh_memcpy_kernel(const uint4* src, uint4* dst, uint64_t n16) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

#include <algorithm>
#include "launch.h"
hipError_t lzh_launch_scan(const uint32_t* csizes, uint64_t nchunks, uint64_t* offsets, uint64_t* total,
                           hipStream_t s) {
    hipLaunchKernelGGL(lzh_scan_kernel, dim3(1), dim3(1024), 0, s, csizes, nchunks, offsets, total);
    return hipGetLastError();
}
hipError_t lzh_launch_pack(const uint8_t* in, uint64_t n_total, uint64_t in_readable, uint64_t chunk_size,
                           const uint8_t* stage, uint64_t stride, const uint32_t* csizes, const uint64_t* offsets,
                           uint8_t* packed, uint64_t packed_cap, uint32_t nchunks, hipStream_t s) {
    if (nchunks == 0) return hipSuccess;
    hipLaunchKernelGGL(lzh_pack_kernel, dim3(nchunks), dim3(256), 0, s, in, n_total, in_readable, chunk_size,
                       stage, stride, csizes, offsets, packed, packed_cap);
    return hipGetLastError();
}
hipError_t lzh_launch_memcpy(const void* src, void* dst, uint64_t n, hipStream_t s) {
    const uint64_t n16 = n / 16;
    if (n16) {
        const uint64_t blocks = std::min<uint64_t>((n16 + 255) / 256, 2048);
        hipLaunchKernelGGL(lzh_memcpy_kernel, dim3((unsigned)blocks), dim3(256), 0, s, (const uint4*)src, (uint4*)dst, n16);
    }
    if (n % 16) {
        hipError_t e = hipMemcpyAsync((uint8_t*)dst + n16 * 16, (const uint8_t*)src + n16 * 16, n % 16,
                                      hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}
