// lzbench_amd/csrc/common.h -- gfx950 device helpers shared by the codec kernels.
//
// Every global access of the codecs goes through raw buffer descriptors
// (__builtin_amdgcn_make_buffer_rsrc): loads past num_records return 0 and stores past it
// are dropped, so a malformed stream or an indexing bug cannot fault the GPU.  The
// descriptor inputs are made provably wave-uniform with readfirstlane (guide T20) so no
// waterfall loops are generated.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LZH_WAVE 64

typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int unii(int v) { return (int)__builtin_amdgcn_readfirstlane((uint32_t)v); }
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    return ((uint64_t)uni((uint32_t)(v >> 32)) << 32) | uni((uint32_t)v);
}

__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    uint64_t a = (uint64_t)p;
    uint32_t lo = uni((uint32_t)a), hi = uni((uint32_t)(a >> 32));
    const void* pu = (const void*)(((uint64_t)hi << 32) | lo);
    return __builtin_amdgcn_make_buffer_rsrc((void*)pu, (short)0, (int)uni(bytes), 0x00020000);
}

__device__ __forceinline__ uint32_t ld_b32(rsrc_t r, int off) { return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0); }
__device__ __forceinline__ uint32_t ld_u8(rsrc_t r, int off) { return __builtin_amdgcn_raw_buffer_load_b8(r, off, 0, 0); }
__device__ __forceinline__ void st_u8(rsrc_t r, int off, uint32_t v) { __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, off, 0, 0); }
__device__ __forceinline__ void st_b32(rsrc_t r, int off, uint32_t v) { __builtin_amdgcn_raw_buffer_store_b32(v, r, off, 0, 0); }
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_b64(rsrc_t r, int off, uint32_t lo, uint32_t hi) {
    const u32x2 v = {lo, hi};
    __builtin_amdgcn_raw_buffer_store_b64(v, r, off, 0, 0);
}

// unaligned little-endian 32-bit read at byte position pos (>= 0) from two aligned dwords
__device__ __forceinline__ uint32_t ld_u32(rsrc_t r, int pos) {
    int a = pos & ~3;
    uint32_t lo = ld_b32(r, a), hi = ld_b32(r, a + 4);
    return __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)pos & 3u);
}
// 40-bit read (bytes pos..pos+4) for LZ4's hash5
__device__ __forceinline__ uint64_t ld_u40(rsrc_t r, int pos) {
    int a = pos & ~3;
    uint32_t s = (uint32_t)pos & 3u;
    uint32_t lo = ld_b32(r, a), hi = ld_b32(r, a + 4);
    uint32_t v = __builtin_amdgcn_alignbyte(hi, lo, s);
    uint32_t b4 = (hi >> (8u * s)) & 0xffu;
    return (uint64_t)v | ((uint64_t)b4 << 32);
}

// v_ffbl_b32: index of the lowest set bit, ~0 for 0 (the hardware result, no zero select)
__device__ __forceinline__ uint32_t ffbl_hw(uint32_t x) {
    uint32_t r;
    asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// index of the first differing byte of two 20-byte windows given their word XORs (20 if none):
// a zero word's v_ffbl is ~0, so the min over "4k + first set byte of word k" picks the first
// nonzero word without a select chain
__device__ __forceinline__ int first_diff20(uint32_t x0, uint32_t x1, uint32_t x2, uint32_t x3, uint32_t x4) {
    const uint32_t f0 = ffbl_hw(x0) >> 3, f1 = (ffbl_hw(x1) >> 3) + 4, f2 = (ffbl_hw(x2) >> 3) + 8,
                   f3 = (ffbl_hw(x3) >> 3) + 12, f4 = (ffbl_hw(x4) >> 3) + 16;
    return (int)min(min(min(f0, f1), min(f2, f3)), min(f4, 20u));
}

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }   // (the lane mask itself: no v_cndmask / v_cmp round trip through a VGPR)
// this lane's bit of a wave-uniform lane mask (the inverse of ballot: one v_cndmask on the SGPR
// pair instead of a 64-bit shift, mask and compare per lane)
__device__ __forceinline__ bool lane_on(uint64_t m) { return __builtin_amdgcn_inverse_ballot_w64(m); }
__device__ __forceinline__ int ffs64(uint64_t m) { return m ? __builtin_ctzll(m) : 64; }
__device__ __forceinline__ uint32_t rdlane(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ int rdlanei(int v, int l) { return (int)__builtin_amdgcn_readlane((uint32_t)v, l); }
// cross-lane gather: value of v held by lane `src` (any lane, 0..63)
__device__ __forceinline__ uint32_t lane_gather(uint32_t v, int src) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}

// Wave-wide inclusive max of x >= 0 by DPP row shifts and row broadcasts (no LDS round trip); with
// x = (member ? end : 0) over lanes whose members' ends increase with the lane, it gives every lane the end
// of the last member at or before it (0: none)
__device__ __forceinline__ int wave_incl_max(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false));   // row_shr:1
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false));   // row_shr:2
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false));   // row_shr:4
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false));   // row_shr:8
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false));   // row_bcast:15 -> rows 1, 3
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false));   // row_bcast:31 -> rows 2, 3
    return x;
}
// the value of lane - 1 (0 in lane 0): DPP wave_shr:1
__device__ __forceinline__ int wave_shr1(int x) { return __builtin_amdgcn_update_dpp(0, x, 0x138, 0xf, 0xf, false); }
// the same by byte address (4 x the source lane; a constant offset can fold into ds_bpermute's offset field)
__device__ __forceinline__ uint32_t lane_gather_b(uint32_t v, int addr) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v);
}
// compiler-level ordering for LDS traffic between lanes of the one wave of a workgroup
// (DS instructions of a wave execute in order in hardware)
__device__ __forceinline__ void wave_lds_fence() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ void wait_vm_but1() { asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); }   // all but the last issued

// Byte-addressed view of a global span through a 4-aligned buffer descriptor: position p
// lives at descriptor offset p + sh (sh = base address mod 4), so chunk bases of any
// alignment are handled with aligned dword accesses only.
struct Bytes {
    rsrc_t r;
    int sh;
    __device__ __forceinline__ void init(const void* p, uint64_t bytes) {
        const uint64_t a = (uint64_t)p;
        sh = (int)uni((uint32_t)a & 3u);
        r = make_rsrc((const void*)(a - (uint64_t)sh), (uint32_t)(bytes + (uint64_t)sh));
    }
    // the same view with its range ending at the dword that holds the last byte: unaligned dword
    // reads of bytes < `bytes` see no zeros, and nothing past that dword (always mapped) is read
    __device__ __forceinline__ void init_dw(const void* p, uint64_t bytes) {
        const uint64_t a = (uint64_t)p;
        sh = (int)uni((uint32_t)a & 3u);
        r = make_rsrc((const void*)(a - (uint64_t)sh), (uint32_t)((bytes + (uint64_t)sh + 3u) & ~3ull));
    }
    __device__ __forceinline__ uint32_t b(int pos) const { return ld_u8(r, pos + sh); }
    __device__ __forceinline__ uint32_t w32(int pos) const { return ld_u32(r, pos + sh); }
    __device__ __forceinline__ uint64_t w40(int pos) const { return ld_u40(r, pos + sh); }
    __device__ __forceinline__ uint32_t b_sc1(int pos) const {   // L1-bypassing byte read
        return __builtin_amdgcn_raw_buffer_load_b8(r, pos + sh, 0, 16);
    }
    __device__ __forceinline__ void st8(int pos, uint32_t v) const { st_u8(r, pos + sh, v); }
    __device__ __forceinline__ void st32_aligned(int pos, uint32_t v) const { st_b32(r, pos + sh, v); }
    __device__ __forceinline__ uint32_t aligned_word(int pos) const { return ld_b32(r, pos + sh); }
};

// dst[d0, d0+len) = src[s0, s0+len) by threads t = 0..nt-1 of the caller's group:
// destination-aligned dword stores for the body (source words assembled with v_alignbyte),
// bytewise head and tail (those may share a dword with a neighbour's bytes).
__device__ __forceinline__ void copy_span(const Bytes& src, int s0, const Bytes& dst, int d0, int len, int t, int nt) {
    if (len <= 0) return;
    const int head = min(len, (4 - ((d0 + dst.sh) & 3)) & 3);
    if (t < head) dst.st8(d0 + t, src.b(s0 + t));
    const int nd = (len - head) >> 2;
    for (int d = t; d < nd; d += nt) {
        const int o = head + 4 * d;
        dst.st32_aligned(d0 + o, src.w32(s0 + o));
    }
    const int tail0 = head + 4 * nd;
    if (t < len - tail0) dst.st8(d0 + tail0 + t, src.b(s0 + tail0 + t));
}

// LDS pointers must carry address space 3: a generic pointer to __shared__ memory compiles to
// flat_load/flat_store (vector-memory pipe, vmcnt waits) instead of ds_read/ds_write.
#define LDSA __attribute__((address_space(3)))
__device__ __forceinline__ void lds_zero16(LDSA uint32_t* p) { p[0] = 0; p[1] = 0; p[2] = 0; p[3] = 0; }

// Emission rings (structs with b / o / flushed / put / flush over a kRing-byte LDS ring, see the
// LZ4 and snappy emission kernels): out[pos, pos+len) = in[src, src+len) for a long literal run.
// The ring is flushed up to pos (its last bytes before pos as byte stores, so no store overlaps
// another), the body goes out as dword stores straight to the staging slot, and the ring takes the
// run's last partial dword so that its next dword flush rewrites those bytes unchanged.
template <int kRing, class OutRing>
__device__ __forceinline__ void bulk_literals(OutRing& R, const Bytes& in, int src, int pos, int len, int lane) {
    R.flush(pos, false, lane);                         // complete dwords before pos
    Bytes ob;
    ob.r = R.o;
    ob.sh = 0;
    const int f = R.flushed;
    if (lane < pos - f) ob.st8(f + lane, ((volatile LDSA uint8_t*)R.b)[(f + lane) & (kRing - 1)]);
    copy_span(in, src, ob, pos, len, lane, LZH_WAVE);
    const int e = pos + len, e4 = e & ~3;
    if (lane < e - e4) R.put(e4 + lane, in.b(src + (e4 - pos) + lane));
    R.flushed = e4;
}

// Block i of a chunk list: plain chunks (bpf == 1: chunk i at i * bs), or the blocks of framed
// layouts (frames of fs bytes, each cut into bpf blocks of bs; the last block of a frame and the
// frames' last one are ragged).  false = past the input (an empty input still has block 0).
__device__ __forceinline__ bool block_span(uint64_t i, uint64_t n_total, uint64_t bs, uint64_t fs, uint32_t bpf,
                                           uint64_t& off, int& n) {
    uint64_t lim = bs;
    if (bpf == 1) {
        off = i * bs;
    } else {
        const uint64_t f = i / bpf, b = i - f * bpf;
        off = f * fs + b * bs;
        lim = min(bs, fs - b * bs);
    }
    if (off >= n_total && !(n_total == 0 && i == 0)) return false;
    n = (int)min(lim, n_total - off);
    return true;
}
