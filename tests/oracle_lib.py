"""tests/oracle_lib.py -- ctypes access to the CPU checkers (TEST INFRASTRUCTURE ONLY).

  oracle/liboracle.so   our C restatement (oracle/*.c)
  oracle/_ref/libref.so the reference lz4 1.9.3 / snappy 1.1.8 compiled from /root/reference
                        (oracle/Makefile `ref`), present wherever it was built
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "liboracle.so")
REF_PATH = os.path.join(ROOT, "oracle", "_ref", "libref.so")
_P, _SZ, _I64 = C.c_void_p, C.c_size_t, C.c_int64
_orc = None
_ref = None


def oracle():
    global _orc
    if _orc is None:
        L = C.CDLL(ORACLE_PATH)
        L.oracle_lz4_compress.restype = C.c_int
        L.oracle_lz4_compress.argtypes = [_P, C.c_int, _P, C.c_int]
        L.oracle_lz4_bound.restype = C.c_int
        L.oracle_lz4_bound.argtypes = [C.c_int]
        L.oracle_lz4_decompress_safe.restype = C.c_int
        L.oracle_lz4_decompress_safe.argtypes = [_P, C.c_int, _P, C.c_int]
        L.oracle_snappy_compress.restype = _SZ
        L.oracle_snappy_compress.argtypes = [_P, _SZ, _P]
        L.oracle_snappy_bound.restype = _SZ
        L.oracle_snappy_bound.argtypes = [_SZ]
        L.oracle_snappy_uncompress.restype = _I64
        L.oracle_snappy_uncompress.argtypes = [_P, _SZ, _P, _SZ]
        for f in (L.oracle_compress_chunks,):
            f.restype = _I64
            f.argtypes = [C.c_int, C.c_int, _P, _SZ, _SZ, _P, _P]
        L.oracle_compress_chunks_mt.restype = _I64
        L.oracle_compress_chunks_mt.argtypes = [C.c_int, C.c_int, _P, _SZ, _SZ, _P, _P, C.c_int]
        L.oracle_decompress_chunks.restype = _I64
        L.oracle_decompress_chunks.argtypes = [C.c_int, _P, _P, _SZ, _SZ, _P]
        L.oracle_lz4f_compress.restype = _I64
        L.oracle_lz4f_compress.argtypes = [_P, _SZ, _P, C.c_int]
        L.oracle_lz4f_decompress.restype = _I64
        L.oracle_lz4f_decompress.argtypes = [_P, _SZ, _P, _SZ]
        L.oracle_lz4f_bound.restype = _SZ
        L.oracle_lz4f_bound.argtypes = [_SZ, C.c_int]
        L.oracle_nvlz4_compress.restype = _I64
        L.oracle_nvlz4_compress.argtypes = [_P, _SZ, _P, C.c_int]
        L.oracle_nvlz4_decompress.restype = _I64
        L.oracle_nvlz4_decompress.argtypes = [_P, _SZ, _P, _SZ]
        L.oracle_xxh32.restype = C.c_uint32
        L.oracle_xxh32.argtypes = [_P, _SZ, C.c_uint32]
        L.oracle_decompress_chunks_mt.restype = _I64
        L.oracle_decompress_chunks_mt.argtypes = [C.c_int, _P, _P, _SZ, _SZ, _P, C.c_int]
        _orc = L
    return _orc


def have_ref() -> bool:
    return os.path.exists(REF_PATH)


def ref():
    global _ref
    if _ref is None:
        L = C.CDLL(REF_PATH)
        L.ref_lz4_version.restype = C.c_int
        L.ref_lz4_compress_fast.restype = C.c_int
        L.ref_lz4_compress_fast.argtypes = [_P, _P, C.c_int, C.c_int, C.c_int]
        L.ref_lz4_decompress_safe.restype = C.c_int
        L.ref_lz4_decompress_safe.argtypes = [_P, _P, C.c_int, C.c_int]
        L.ref_snappy_compress.restype = _SZ
        L.ref_snappy_compress.argtypes = [_P, _SZ, _P]
        L.ref_snappy_uncompress.restype = C.c_int
        L.ref_snappy_uncompress.argtypes = [_P, _SZ, _P]
        L.ref_compress_chunks.restype = _I64
        L.ref_compress_chunks.argtypes = [C.c_int, C.c_int, _P, _SZ, _SZ, _P, _P]
        L.ref_decompress_chunks.restype = _I64
        L.ref_decompress_chunks.argtypes = [C.c_int, _P, _P, _SZ, _SZ, _P]
        L.ref_compress_chunks_mt.restype = _I64
        L.ref_compress_chunks_mt.argtypes = [C.c_int, C.c_int, _P, _SZ, _SZ, _P, _P, C.c_int]
        L.ref_decompress_chunks_mt.restype = _I64
        L.ref_decompress_chunks_mt.argtypes = [C.c_int, _P, _P, _SZ, _SZ, _P, C.c_int]
        L.ref_zstd_compress.restype = _I64
        L.ref_zstd_compress.argtypes = [_P, _SZ, _P, _SZ, C.c_int]
        L.ref_zstd_decompress.restype = _I64
        L.ref_zstd_decompress.argtypes = [_P, _SZ, _P, _SZ]
        L.ref_zstd_version.restype = C.c_int
        L.ref_zstd_compress_checksum.restype = _I64
        L.ref_zstd_compress_checksum.argtypes = [_P, _SZ, _P, _SZ, C.c_int]
        L.ref_lz4f_compress.restype = _I64
        L.ref_lz4f_compress.argtypes = [_P, _SZ, _P, _SZ, C.c_int]
        L.ref_lz4f_decompress.restype = _I64
        L.ref_lz4f_decompress.argtypes = [_P, _SZ, _P, _SZ]
        L.ref_lz4f_bound.restype = _SZ
        L.ref_lz4f_bound.argtypes = [_SZ, C.c_int]
        _ref = L
    return _ref


CODEC_ID = {"lz4": 0, "lz4fast": 0, "snappy": 1, "zstd": 2, "lz4f": 3, "nvlz4": 4}   # zstd decode: reference build only


def lz4_compress(data: np.ndarray, acc: int = 1) -> bytes:
    L = oracle()
    out = np.zeros(L.oracle_lz4_bound(len(data)) + 64, np.uint8)
    r = L.oracle_lz4_compress(data.ctypes.data, len(data), out.ctypes.data, acc)
    return out[:r].tobytes()


def snappy_compress(data: np.ndarray) -> bytes:
    L = oracle()
    out = np.zeros(L.oracle_snappy_bound(len(data)) + 64, np.uint8)
    r = L.oracle_snappy_compress(data.ctypes.data, len(data), out.ctypes.data)
    return out[:r].tobytes()


def compress_chunks(data: np.ndarray, codec: str, chunk: int, level: int = 1, use_ref=None, threads: int = 0):
    """lzbench_compress over uniform chunks with the CPU checker. Returns (packed, csizes).
    use_ref None: the restatement for lz4/snappy, the reference build for zstd when present
    (the restatement covers zstd's fast-strategy levels only: oracle/zstd1_oracle.c)."""
    n = len(data)
    k = max((n + chunk - 1) // chunk, 1)
    out = np.zeros(n + n // 6 + 16384 + 64 * k + 64, np.uint8)
    cs = np.zeros(k, np.uint64)
    c = CODEC_ID[codec]
    lvl = level if codec in ("lz4fast", "zstd", "lz4f", "nvlz4") else (1 if codec == "lz4" else 0)
    if use_ref is None:
        use_ref = codec == "zstd" and have_ref()
    if use_ref:
        L = ref()
        tot = (L.ref_compress_chunks_mt(c, lvl, data.ctypes.data, n, chunk, out.ctypes.data, cs.ctypes.data, threads)
               if threads else L.ref_compress_chunks(c, lvl, data.ctypes.data, n, chunk, out.ctypes.data, cs.ctypes.data))
    else:
        L = oracle()
        tot = (L.oracle_compress_chunks_mt(c, lvl, data.ctypes.data, n, chunk, out.ctypes.data, cs.ctypes.data, threads)
               if threads else L.oracle_compress_chunks(c, lvl, data.ctypes.data, n, chunk, out.ctypes.data, cs.ctypes.data))
    return out[:tot].copy(), cs


def decompress_chunks(packed: np.ndarray, csizes: np.ndarray, n: int, codec: str, chunk: int, use_ref=False, threads=0):
    out = np.zeros(n + 64, np.uint8)
    c = CODEC_ID[codec]
    packed = np.ascontiguousarray(packed)
    cs = np.ascontiguousarray(csizes, dtype=np.uint64)
    if use_ref or codec == "zstd":   # (lz4f / nvlz4: the restatement unless use_ref)
        L = ref()
        r = (L.ref_decompress_chunks_mt(c, packed.ctypes.data, cs.ctypes.data, n, chunk, out.ctypes.data, threads)
             if threads else L.ref_decompress_chunks(c, packed.ctypes.data, cs.ctypes.data, n, chunk, out.ctypes.data))
    else:
        L = oracle()
        r = (L.oracle_decompress_chunks_mt(c, packed.ctypes.data, cs.ctypes.data, n, chunk, out.ctypes.data, threads)
             if threads else L.oracle_decompress_chunks(c, packed.ctypes.data, cs.ctypes.data, n, chunk, out.ctypes.data))
    return r, out[:n]
