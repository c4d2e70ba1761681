"""CPU: AddressSanitizer + UndefinedBehaviorSanitizer runs of the host C/C++ code:
the oracle restatements and the corpus generator (tests/asan/oracle_asan_main.c: chunk loops,
multi-threaded variants, round trips, malformed-stream rejection) and the lzbench-style CLI driver
(its CPU rows: option parsing, chunk loop, -j / -m / -o / -x paths).  Device code is not
sanitized (GPU sanitizers are not available on this pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")


def test_oracle_and_datagen_under_asan_ubsan(tmp_path):
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    exe = tmp_path / "oracle_asan"
    src = [os.path.join(ROOT, "tests", "asan", "oracle_asan_main.c")] + \
          [os.path.join(ROOT, "oracle", f) for f in ("lz4_oracle.c", "snappy_oracle.c", "zstd1_oracle.c", "chunks_oracle.c",
                                                     "frame_oracle.c")] + \
          [os.path.join(ROOT, "lzbench_amd", "csrc", "datagen.c")]
    subprocess.run(["gcc", "-std=gnu11", "-pthread", *SAN, "-o", str(exe), *src, "-lm"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=ENV, timeout=600)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr


def test_cli_driver_under_asan_ubsan(tmp_path):
    hipcc = "/opt/rocm/bin/hipcc"
    lib = os.path.join(ROOT, "lzbench_amd", "liblzbench_hip.so")
    if not (os.path.exists(hipcc) and os.path.exists(lib)):
        pytest.skip("hipcc or liblzbench_hip.so missing")
    exe = tmp_path / "lzbench_hip_asan"
    subprocess.run([hipcc, "-std=c++17", "-fno-gpu-sanitize", *SAN, "-o", str(exe),
                    os.path.join(ROOT, "lzbench_amd", "driver", "lzbench_hip_main.cpp"),
                    "-L" + os.path.dirname(lib), "-llzbench_hip", "-ldl", "-Wl,-rpath," + os.path.dirname(lib)],
                   check=True)
    import lzbench_amd as L
    f1, f2 = tmp_path / "a.bin", tmp_path / "b.bin"
    L.datagen("text", 700_000, seed=1).tofile(f1)
    L.datagen("json", 300_001, seed=2).tofile(f2)
    runs = [["-elz4/lz4fast,3,17", "-b64", "-t0,0", "-x", str(f1)],
            ["-elz4", "-b128", "-t0,0", "-j", "-o4", str(f1), str(f2)],
            ["-elz4fast,5", "-b64", "-t0,0", "-m1", "-p3", "-c4", str(f1)],
            ["-l"]]
    for args in runs:
        r = subprocess.run([str(exe), *args], capture_output=True, text=True, env=ENV, timeout=300)
        assert r.returncode == 0, (args, r.stdout, r.stderr)
        assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, (args, r.stderr)
