"""Staleness guard of the roofline's traffic figures (round-5 verdict item 5): bench.py reports a committed PMC
profile's HBM bytes only for the machine code that profile measured.  CPU: the library's code objects are read,
not run."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lzbench_amd import kernel_hash  # noqa: E402

LIB = os.path.join(ROOT, "lzbench_amd", "liblzbench_hip.so")


@pytest.fixture(scope="module")
def hashes():
    if not os.path.exists(LIB):
        pytest.skip("liblzbench_hip.so not built")
    return kernel_hash.kernel_hashes(LIB)


def test_every_bench_kernel_has_a_code_hash(hashes):
    for k in ("lzh_lz4_parse_kernel", "lzh_lz4_emit_kernel", "lzh_scan_kernel", "lzh_pack_kernel",
              "lzh_decompress_v2_kernel", "lzh_decompress_w8k_kernel", "lzh_snappy_parse_kernel",
              "lzh_zstd_match_kernel", "lzh_zstd_entropy_kernel", "lzh_zstd_seq_kernel"):
        assert len(hashes.get(k, "")) == 16, k
    assert kernel_hash.kernel_hashes(LIB) == hashes          # deterministic


def test_traffic_only_for_the_profiled_code(hashes, tmp_path, monkeypatch):
    import bench
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "_HASHES", dict(hashes))
    (tmp_path / "profiles").mkdir()
    k = "lzh_lz4_parse_kernel"
    prof = {"workload_key": "w", "kernels": {k: {"traffic_bytes_per_dispatch": 123.0, "kernel_hash": hashes[k]}}}
    (tmp_path / "profiles" / "traffic_a.json").write_text(json.dumps(prof))
    assert bench.traffic_for(k, "w") == (123, None)
    assert bench.traffic_for(k, "other")[0] is None
    prof["kernels"][k]["kernel_hash"] = "0" * 16               # measured other machine code
    (tmp_path / "profiles" / "traffic_a.json").write_text(json.dumps(prof))
    v, why = bench.traffic_for(k, "w")
    assert v is None and "other code" in why
    del prof["kernels"][k]["kernel_hash"]                       # a profile from before the hashes
    (tmp_path / "profiles" / "traffic_a.json").write_text(json.dumps(prof))
    assert bench.traffic_for(k, "w")[0] is None


def test_bench_reads_the_loaded_library(hashes, monkeypatch):
    """bench.py hashes the library lzbench_amd loads (LIB_PATH), not a copy"""
    import bench
    monkeypatch.setattr(bench, "_HASHES", None)
    assert bench._loaded_hashes() == hashes
