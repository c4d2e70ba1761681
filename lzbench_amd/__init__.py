"""lzbench_amd -- host-side mirror of lzbench's compressor_desc_t table and chunk loop for the
MI355X (gfx950) LZ4 / snappy codecs of liblzbench_hip.so.

Reference interface mirrored here:
  * compressor_desc_t rows ........ /root/reference/_lzbench/lzbench.h:113-129, :140-219
  * lzbench_compress / _decompress  /root/reference/_lzbench/lzbench.cpp:266-298 / :301-329
    (raw-store rule clen <= 0 || clen == part, contiguous packing, compr_sizes[])
  * GET_COMPRESS_BOUND ............ /root/reference/_lzbench/lzbench.h:17

Everything here is a thin ctypes layer over the C-ABI in include/lzbench_hip.h; the codec
work runs in the HIP kernels of lzbench_amd/csrc.  There is no CPU fallback: if the shared
library is missing the import of any codec entry point raises ExtensionMissing.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

__all__ = [
    "ExtensionMissing", "lib", "CODECS", "COMP_DESC", "CompressorDesc", "find_compressor",
    "compress_chunks", "decompress_chunks", "chunk_sizes_for", "datagen", "DeviceCodec",
    "LZH_CODEC_LZ4", "LZH_CODEC_SNAPPY", "LZH_CODEC_MEMCPY", "LZH_CODEC_ZSTD", "LZH_CODEC_LZ4F", "LZH_CODEC_NVLZ4",
    "LZ4F_BLOCK_CHECKSUM", "LZ4F_CONTENT_CHECKSUM", "LZ4F_CONTENT_SIZE", "LZ4F_LINKED", "PAD_SIZE",
    "get_compress_bound",
]

_HERE = os.path.dirname(os.path.abspath(__file__))
# LZH_LIB: an alternative in-tree build of the same library (kernel experiments; tools/exp_build.sh)
LIB_PATH = os.environ.get("LZH_LIB") or os.path.join(_HERE, "liblzbench_hip.so")
DATAGEN_PATH = os.path.join(_HERE, "libdatagen.so")

LZH_CODEC_LZ4, LZH_CODEC_SNAPPY, LZH_CODEC_MEMCPY, LZH_CODEC_ZSTD, LZH_CODEC_LZ4F, LZH_CODEC_NVLZ4 = 0, 1, 2, 3, 4, 5
CODECS = {"lz4": LZH_CODEC_LZ4, "lz4fast": LZH_CODEC_LZ4, "snappy": LZH_CODEC_SNAPPY, "memcpy": LZH_CODEC_MEMCPY,
          "zstd": LZH_CODEC_ZSTD, "zstd_fast": LZH_CODEC_ZSTD, "lz4frame": LZH_CODEC_LZ4F,
          "nvcomp_lz4": LZH_CODEC_NVLZ4}
# LZ4 frame parameters (include/lzbench_hip.h LZH_LZ4F_*): level = bsid | flags | acceleration << 8
LZ4F_BLOCK_CHECKSUM, LZ4F_CONTENT_CHECKSUM, LZ4F_CONTENT_SIZE, LZ4F_LINKED = 0x10, 0x20, 0x40, 0x80
# codecs whose level is passed through as is (the others: 1 for lz4 = LZ4_compress_default, 0)
_LEVELED = ("lz4fast", "zstd", "zstd_fast", "lz4frame", "nvcomp_lz4")
PAD_SIZE = 16 * 1024          # lzbench.h:14


def get_compress_bound(n: int) -> int:
    """GET_COMPRESS_BOUND (lzbench.h:17)."""
    return n + n // 6 + PAD_SIZE


class ExtensionMissing(RuntimeError):
    """liblzbench_hip.so is not built (run __graft_entry__.build())."""


_P = C.c_void_p
_SZ = C.c_size_t
_I64 = C.c_int64
_lib = None
_dg = None

# exported symbols and their signatures (restype, argtypes) -- kept in sync with
# include/lzbench_hip.h; tests/test_abi.py checks every header declaration is here and loads
_COMPRESS_FUNC = (_I64, [_P, _SZ, _P, _SZ, _SZ, _SZ, _P])
SIGNATURES = {
    "lzbench_hip_lz4_init": (_P, [_SZ, _SZ, _SZ]),
    "lzbench_hip_snappy_init": (_P, [_SZ, _SZ, _SZ]),
    "lzbench_hip_memcpy_init": (_P, [_SZ, _SZ, _SZ]),
    "lzbench_hip_zstd_init": (_P, [_SZ, _SZ, _SZ]),
    "lzbench_hip_lz4frame_init": (_P, [_SZ, _SZ, _SZ]),
    "lzbench_hip_nvcomp_lz4_init": (_P, [_SZ, _SZ, _SZ]),
    "lzbench_hip_lz4frame_compress": _COMPRESS_FUNC,
    "lzbench_hip_lz4frame_decompress": _COMPRESS_FUNC,
    "lzbench_hip_nvcomp_lz4_compress": _COMPRESS_FUNC,
    "lzbench_hip_nvcomp_lz4_decompress": _COMPRESS_FUNC,
    "lzbench_hip_zstd_compress": _COMPRESS_FUNC,
    "lzbench_hip_zstd_decompress": _COMPRESS_FUNC,
    "lzbench_hip_deinit": (None, [_P]),
    "lzbench_hip_lz4_compress": _COMPRESS_FUNC,
    "lzbench_hip_lz4fast_compress": _COMPRESS_FUNC,
    "lzbench_hip_lz4_decompress": _COMPRESS_FUNC,
    "lzbench_hip_snappy_compress": _COMPRESS_FUNC,
    "lzbench_hip_snappy_decompress": _COMPRESS_FUNC,
    "lzbench_hip_memcpy": _COMPRESS_FUNC,
    "lzbench_hip_compress_batch": (_I64, [_P, _P, C.c_int, _P, _SZ, _P, _SZ, _SZ, _P]),
    "lzbench_hip_decompress_batch": (_I64, [_P, _P, _P, C.c_int, _P, _SZ, _SZ, _SZ, _P]),
    "lzh_stage_stride": (_SZ, [C.c_int, _SZ]),
    "lzh_max_packed_bytes": (_SZ, [C.c_int, _SZ, _SZ]),
    "lzh_compress_temp_bytes": (_SZ, [C.c_int, _SZ, _SZ]),
    "lzh_decompress_temp_bytes": (_SZ, [C.c_int, _SZ, _SZ]),
    "lzh_num_chunks": (_SZ, [_SZ, _SZ]),
    "lzh_level_supported": (C.c_int, [C.c_int, C.c_int, _SZ]),
    "lzh_debug_plan": (C.c_int, [_SZ, _SZ, _SZ, C.c_int, _P, C.c_int]),
    "lzh_debug_gather_order": (C.c_int, [_SZ, _P, _P, _P]),
    "lzh_compress_async": (C.c_int, [C.c_int, C.c_int, _P, _SZ, _SZ, _SZ, _P, _SZ, _P, _P, _P, _SZ, _P]),
    "lzh_decompress_async": (C.c_int, [C.c_int, _P, _SZ, _P, _P, _SZ, _SZ, _P, _P, _P, _SZ, _P]),
    "lzh_compress_kernel_only": (C.c_int, [C.c_int, C.c_int, _P, _SZ, _SZ, _SZ, _P, _P, _P]),
    "lzh_compress_kernel_stage": (C.c_int, [C.c_int, C.c_int, C.c_int, _P, _SZ, _SZ, _SZ, _P, _P, _P]),
    "lzh_compress_finish_async": (C.c_int, [C.c_int, _P, _SZ, _SZ, _SZ, _P, _P, _P, _SZ, _P, _P]),
    "lzh_datagen": (_SZ, [C.c_int, C.c_uint64, _P, _SZ]),
    "lzh_version": (C.c_char_p, []),
}


def lib():
    """The loaded C-ABI library (raises ExtensionMissing if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ExtensionMissing(f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            # (an older experiment build named by LZH_LIB may lack the newest debug entry points)
            if os.environ.get("LZH_LIB") and name.startswith("lzh_debug") and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def datagen(kind: str | int, n: int, seed: int = 12345, offset: int = 0) -> np.ndarray:
    """Synthetic corpus: random / text / json / mixed / binary.  offset (a multiple
    of 16 MiB): bytes [offset, offset + n) of the same corpus -- a rank's share of a multi-GiB input
    (the corpus is generated in independent 16 MiB segments, so a share needs no prefix)."""
    global _dg
    kinds = {"random": 0, "text": 1, "json": 2, "mixed": 3, "binary": 4}
    k = kinds[kind] if isinstance(kind, str) else int(kind)
    if _dg is None:
        if not os.path.exists(DATAGEN_PATH):
            raise ExtensionMissing(f"{DATAGEN_PATH} not found")
        _dg = C.CDLL(DATAGEN_PATH)
        _dg.lzb_datagen.restype = _SZ
        _dg.lzb_datagen.argtypes = [C.c_int, C.c_uint64, _P, _SZ]
        _dg.lzb_datagen_at.restype = _SZ
        _dg.lzb_datagen_at.argtypes = [C.c_int, C.c_uint64, _P, _SZ, _SZ]
    if offset % (16 << 20):
        raise ValueError("datagen offset must be a multiple of 16 MiB")
    buf = np.empty(max(n, 1), dtype=np.uint8)
    if _dg.lzb_datagen_at(k, C.c_uint64(seed), buf.ctypes.data, offset, n) != n:
        raise ValueError(f"bad corpus kind {kind}")
    return buf[:n]


@dataclass(frozen=True)
class CompressorDesc:
    """One row of lzbench's comp_desc[] (lzbench.h:117-129); function fields name C symbols."""
    name: str
    version: str
    first_level: int
    last_level: int
    additional_param: int
    max_block_size: int
    compress: Optional[str]
    decompress: Optional[str]
    init: Optional[str]
    deinit: Optional[str]
    compress_batch: Optional[str] = None
    decompress_batch: Optional[str] = None


# index 0 stays memcpy (lzbench.cpp:609, :695); the GPU rows replace cudaMemcpy / nvcomp_lz4
# (lzbench.h:217-218) and add bit-exact lz4 / lz4fast / snappy rows.
COMP_DESC = (
    CompressorDesc("memcpy", "", 0, 0, 0, 0, None, None, None, None),
    CompressorDesc("hipMemcpy", "", 0, 0, 1, 0, "lzbench_hip_memcpy", "lzbench_hip_memcpy",
                   "lzbench_hip_memcpy_init", "lzbench_hip_deinit",
                   "lzbench_hip_compress_batch", "lzbench_hip_decompress_batch"),
    CompressorDesc("hip_lz4", "1.9.3", 0, 0, 1, 0, "lzbench_hip_lz4_compress", "lzbench_hip_lz4_decompress",
                   "lzbench_hip_lz4_init", "lzbench_hip_deinit",
                   "lzbench_hip_compress_batch", "lzbench_hip_decompress_batch"),
    CompressorDesc("hip_lz4fast", "1.9.3", 1, 99, 1, 0, "lzbench_hip_lz4fast_compress", "lzbench_hip_lz4_decompress",
                   "lzbench_hip_lz4_init", "lzbench_hip_deinit",
                   "lzbench_hip_compress_batch", "lzbench_hip_decompress_batch"),
    CompressorDesc("hip_snappy", "2020-07-11", 0, 0, 1, 0, "lzbench_hip_snappy_compress",
                   "lzbench_hip_snappy_decompress", "lzbench_hip_snappy_init", "lzbench_hip_deinit",
                   "lzbench_hip_compress_batch", "lzbench_hip_decompress_batch"),
    # zstd / zstd_fast rows (lzbench.h:209-210) restricted to the fast-strategy levels
    CompressorDesc("hip_zstd", "1.5.2", 1, 2, 1, 0, "lzbench_hip_zstd_compress", "lzbench_hip_zstd_decompress",
                   "lzbench_hip_zstd_init", "lzbench_hip_deinit",
                   "lzbench_hip_compress_batch", "lzbench_hip_decompress_batch"),
    CompressorDesc("hip_zstd_fast", "1.5.2", -5, -1, 1, 0, "lzbench_hip_zstd_compress", "lzbench_hip_zstd_decompress",
                   "lzbench_hip_zstd_init", "lzbench_hip_deinit",
                   "lzbench_hip_compress_batch", "lzbench_hip_decompress_batch"),
    # framed formats: an LZ4 frame per chunk (level = LZH_LZ4F_PARAMS), the nvcomp_lz4 row's container
    # (lzbench.h:218, levels 0..5 = chunks of 32 KiB << level)
    CompressorDesc("hip_lz4frame", "1.9.3", 4, 7, 1, 0, "lzbench_hip_lz4frame_compress",
                   "lzbench_hip_lz4frame_decompress", "lzbench_hip_lz4frame_init", "lzbench_hip_deinit",
                   "lzbench_hip_compress_batch", "lzbench_hip_decompress_batch"),
    CompressorDesc("hip_nvcomp_lz4", "1.2.2", 0, 5, 1, 0, "lzbench_hip_nvcomp_lz4_compress",
                   "lzbench_hip_nvcomp_lz4_decompress", "lzbench_hip_nvcomp_lz4_init", "lzbench_hip_deinit",
                   "lzbench_hip_compress_batch", "lzbench_hip_decompress_batch"),
)


def find_compressor(name: str) -> CompressorDesc:
    """Name lookup as in lzbench_test_with_params (lzbench.cpp:492-530); plain codec names
    (lz4, lz4fast, snappy) resolve to their GPU rows."""
    for d in COMP_DESC:
        if d.name == name or d.name == "hip_" + name:
            return d
    raise KeyError(f"{name} NOT FOUND")


def chunk_sizes_for(n: int, chunk_size: int) -> np.ndarray:
    """lzbench_test's chunk list for one file (lzbench.cpp:366-373)."""
    k = (n + chunk_size - 1) // chunk_size
    cs = np.full(k, chunk_size, dtype=np.uint64)
    if k and n % chunk_size:
        cs[-1] = n % chunk_size
    return cs


def _as_u8(a) -> np.ndarray:
    if isinstance(a, (bytes, bytearray, memoryview)):
        return np.frombuffer(bytes(a), dtype=np.uint8)
    a = np.ascontiguousarray(a)
    return a.view(np.uint8).reshape(-1)


class _Row:
    """An init'ed GPU row (workmem owner)."""

    def __init__(self, codec: str, chunk_size: int, level: int = 0, ngpus: int = 1):
        L = lib()
        base = {"memcpy": "memcpy", "snappy": "snappy", "zstd": "zstd", "zstd_fast": "zstd", "lz4frame": "lz4frame",
                "nvcomp_lz4": "nvcomp_lz4"}.get(codec, "lz4")
        self.desc = find_compressor("hipMemcpy" if codec == "memcpy" else codec)
        self.wm = getattr(L, f"lzbench_hip_{base}_init")(chunk_size, level, ngpus)
        if not self.wm:
            raise RuntimeError("lzbench_hip init failed (no HIP device?)")
        self.level = level

    def close(self):
        if self.wm:
            lib().lzbench_hip_deinit(self.wm)
            self.wm = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def _row_level(codec: str, level: int) -> int:
    """The level argument lzbench passes for the row: lz4fast acceleration, zstd level (zstd_fast
    rows are negative), 1 for lz4 (LZ4_compress_default), 0 for snappy; size_t on the wire."""
    if codec in _LEVELED:
        return level & 0xFFFFFFFFFFFFFFFF
    return 1 if codec == "lz4" else 0


def compress_chunks(data, codec: str = "lz4", chunk_size: int = 65536, level: int = 0, ngpus: int = 1,
                    chunk_sizes=None) -> Tuple[np.ndarray, np.ndarray]:
    """lzbench_compress over the chunk list on the GPU(s). Returns (packed bytes, compr_sizes)."""
    src = _as_u8(data)
    cs = np.ascontiguousarray(chunk_sizes if chunk_sizes is not None else chunk_sizes_for(len(src), chunk_size),
                              dtype=np.uint64)
    out = np.zeros(get_compress_bound(len(src)) + 64, dtype=np.uint8)
    compr = np.zeros(len(cs), dtype=np.uint64)
    lvl = _row_level(codec, level)
    with _Row(codec, chunk_size, lvl, ngpus) as row:
        total = lib().lzbench_hip_compress_batch(src.ctypes.data, cs.ctypes.data, len(cs), out.ctypes.data,
                                                 len(out), compr.ctypes.data, lvl, ngpus, row.wm)
    if total <= 0 and len(src) > 0:
        raise RuntimeError(f"compress_batch failed ({total})")
    return out[:total].copy(), compr


def decompress_chunks(packed, compr_sizes, n: int, codec: str = "lz4", chunk_size: int = 65536, ngpus: int = 1,
                      chunk_sizes=None) -> np.ndarray:
    """lzbench_decompress over the chunk list on the GPU(s). Raises on malformed chunks."""
    src = _as_u8(packed)
    cs = np.ascontiguousarray(chunk_sizes if chunk_sizes is not None else chunk_sizes_for(n, chunk_size),
                              dtype=np.uint64)
    comp = np.ascontiguousarray(compr_sizes, dtype=np.uint64)
    out = np.zeros(n + PAD_SIZE, dtype=np.uint8)
    with _Row(codec, chunk_size, 0, ngpus) as row:
        total = lib().lzbench_hip_decompress_batch(src.ctypes.data, comp.ctypes.data, cs.ctypes.data, len(cs),
                                                   out.ctypes.data, len(out), 0, ngpus, row.wm)
    if total != n:
        raise RuntimeError(f"decompress_batch failed ({total})")
    return out[:n]


class DeviceCodec:
    """Device-resident batched codec on HBM tensors (include/lzbench_hip.h layer 3).

    Buffers are torch uint8 CUDA tensors; work is queued on torch's current stream, so
    torch.cuda.Event pairs on that stream time it.
    """

    def __init__(self, codec: str, n: int, chunk_size: int, level: int = 0, device=None):
        import torch
        self.torch = torch
        self.codec = CODECS[codec]
        self.level = level if codec in _LEVELED else (1 if codec == "lz4" else 0)
        self.n, self.chunk_size = n, chunk_size
        L = lib()
        self.k = L.lzh_num_chunks(n, chunk_size)
        dev = device or torch.device("cuda", torch.cuda.current_device())
        u8 = dict(dtype=torch.uint8, device=dev)
        self.max_packed = L.lzh_max_packed_bytes(self.codec, n, chunk_size)
        self.packed = torch.empty(self.max_packed + 64, **u8)
        self.csizes = torch.empty(self.k, dtype=torch.int32, device=dev)
        self.offsets = torch.empty(self.k + 1, dtype=torch.int64, device=dev)
        self.status = torch.empty(self.k, dtype=torch.int32, device=dev)
        self.ctemp = torch.empty(max(L.lzh_compress_temp_bytes(self.codec, n, chunk_size), 256), **u8)
        self.dtemp = torch.empty(max(L.lzh_decompress_temp_bytes(self.codec, n, chunk_size), 256), **u8)
        self.out = torch.empty(n + 64, **u8)

    def _stream(self):
        return self.torch.cuda.current_stream().cuda_stream

    def compress(self, d_in, in_readable: Optional[int] = None) -> None:
        rc = lib().lzh_compress_async(self.codec, self.level, d_in.data_ptr(), self.n,
                                      in_readable if in_readable is not None else d_in.numel(), self.chunk_size,
                                      self.packed.data_ptr(), self.packed.numel(), self.csizes.data_ptr(),
                                      self.offsets.data_ptr(), self.ctemp.data_ptr(), self.ctemp.numel(),
                                      self._stream())
        if rc:
            raise RuntimeError(f"lzh_compress_async failed ({rc})")

    def compress_kernel_only(self, d_in) -> None:
        rc = lib().lzh_compress_kernel_only(self.codec, self.level, d_in.data_ptr(), self.n, d_in.numel(),
                                            self.chunk_size, self.ctemp.data_ptr(), self.csizes.data_ptr(),
                                            self._stream())
        if rc:
            raise RuntimeError(f"lzh_compress_kernel_only failed ({rc})")

    def compress_stage(self, d_in, stage_mask: int) -> None:
        """One stage of compress_kernel_only (1 = parse kernel, 2 = LZ4 emission kernel)."""
        rc = lib().lzh_compress_kernel_stage(self.codec, self.level, stage_mask, d_in.data_ptr(), self.n, d_in.numel(),
                                             self.chunk_size, self.ctemp.data_ptr(), self.csizes.data_ptr(),
                                             self._stream())
        if rc:
            raise RuntimeError(f"lzh_compress_kernel_stage failed ({rc})")

    def compress_finish(self, d_in) -> None:
        rc = lib().lzh_compress_finish_async(self.codec, d_in.data_ptr(), self.n, d_in.numel(), self.chunk_size,
                                             self.ctemp.data_ptr(), self.csizes.data_ptr(), self.packed.data_ptr(),
                                             self.packed.numel(), self.offsets.data_ptr(), self._stream())
        if rc:
            raise RuntimeError(f"lzh_compress_finish_async failed ({rc})")

    def decompress(self, packed=None, csizes=None, offsets=None) -> None:
        packed = self.packed if packed is None else packed
        csizes = self.csizes if csizes is None else csizes
        rc = lib().lzh_decompress_async(self.codec, packed.data_ptr(), packed.numel(), csizes.data_ptr(),
                                        offsets.data_ptr() if offsets is not None else None, self.n,
                                        self.chunk_size, self.out.data_ptr(), self.status.data_ptr(),
                                        self.dtemp.data_ptr(), self.dtemp.numel(), self._stream())
        if rc:
            raise RuntimeError(f"lzh_decompress_async failed ({rc})")

    def packed_total(self) -> int:
        return int(self.offsets[self.k].item())
