"""The lzbench-compatible CLI driver (lzbench_amd/lzbench_hip): chunk loop, verification and
output formats like the reference lzbench (lzbench.cpp:73-238, :266-476)."""
import os
import subprocess

import numpy as np
import pytest

import lzbench_amd as L
import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "lzbench_amd", "lzbench_hip")


def run(args, env=None):
    r = subprocess.run([EXE] + args, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr
    return r.stdout


def rows(out):
    res = {}
    for line in out.splitlines():
        if "MB/s" in line or "ERROR" in line:
            name = line[:23].strip()
            parts = line[23:].split()
            res[name] = parts
    return res


@pytest.fixture(scope="module")
def sample(tmp_path_factory):
    d = L.datagen("text", 3 * 65536 + 4321, seed=21)
    p = tmp_path_factory.mktemp("drv") / "sample.txt"
    p.write_bytes(d.tobytes())
    return str(p), d


def test_usage_and_list():
    r = subprocess.run([EXE], capture_output=True, text=True)
    assert r.returncode == 1 and "usage" in r.stderr
    out = run(["-l"])
    assert "hip_lz4 1.9.3" in out and "hip_snappy 2020-07-11" in out


def test_cpu_rows_chunk_loop(sample):
    path, data = sample
    out = run(["-elz4", "-b64", "-t0,0", "-i1,1", path])
    r = rows(out)
    assert "memcpy" in r                                  # implicit memcpy row first
    lz4 = [k for k in r if k.startswith("lz4 ")]
    assert lz4, out
    packed, cs = O.compress_chunks(data, "lz4", 65536)
    assert int(r[lz4[0]][4]) == len(packed)              # Compr. size column
    assert "ERROR" not in out


def test_csv_format(sample):
    path, _ = sample
    out = run(["-elz4", "-b64", "-t0,0", "-o4", path])
    lines = [l for l in out.splitlines() if l]
    assert lines[0].startswith("Compressor name,Compression speed")
    assert any(l.startswith("lz4 ") for l in lines[1:])


@pytest.mark.gpu
def test_gpu_rows_match_reference_sizes(sample):
    path, data = sample
    out = run(["-ehip_lz4/hip_snappy/hip_lz4fast,3/hipMemcpy", "-b64", "-t0,0", "-i2,2", path])
    r = rows(out)
    assert "ERROR" not in out, out
    exp = {"hip_lz4": O.compress_chunks(data, "lz4", 65536),
           "hip_snappy": O.compress_chunks(data, "snappy", 65536),
           "hip_lz4fast": O.compress_chunks(data, "lz4fast", 65536, 3)}
    for name, (packed, _) in exp.items():
        key = [k for k in r if k.startswith(name + " ")]
        assert key, (name, out)
        assert int(r[key[0]][4]) == len(packed), (name, out)
    assert any(k.startswith("hipMemcpy") for k in r)


@pytest.mark.gpu
def test_gpu_rows_joined_multi_file(tmp_path):
    a = L.datagen("json", 100_001, seed=1)
    b = L.datagen("text", 70_003, seed=2)
    pa, pb = tmp_path / "a.json", tmp_path / "b.txt"
    pa.write_bytes(a.tobytes())
    pb.write_bytes(b.tobytes())
    out = run(["-ehip_lz4", "-b64", "-t0,0", "-j", str(pa), str(pb)])
    r = rows(out)
    key = [k for k in r if k.startswith("hip_lz4")][0]
    exp = len(O.compress_chunks(a, "lz4", 65536)[0]) + len(O.compress_chunks(b, "lz4", 65536)[0])
    assert int(r[key][4]) == exp and "ERROR" not in out
