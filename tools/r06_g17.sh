# round 6 call 17: zstd match finder's collision groups bit-sliced as the LZ4 kernel's (no per-lane 64-bit select
# per bit), count_bwd's stop mask from single compares, the redundant valid test in prev (zstd, LZ4): zstd compress
# tests + 1 GiB zstd line bit-exact, LZ4 parity, A/B against the head
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_r; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --codec zstd --chunk-kib 128 --corpus mixed > $O/bench_zstd.json 2> $O/bench_zstd.err || { tail $O/bench_zstd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_zstd.json'));print('zstd', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/bench_north.json 2> $O/bench_north.err || { tail $O/bench_north.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_north.json'));print('north', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_zstd_compress.py tests/test_gpu_parity.py -k "zstd or lz4 or LZ4" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
PROF_ARGS="--codec zstd --level 1 --chunk-kib 128" AB_CORPORA="mixed text" AB_ROUNDS=3 timeout -k 10 500 bash tools/ab.sh head base > $O/abz.log 2>&1 || { tail $O/abz.log; exit 1; }
cat $O/abz.log
AB_CORPORA="text" AB_ROUNDS=2 timeout -k 10 300 bash tools/ab.sh head base > $O/ablz.log 2>&1 || { tail $O/ablz.log; exit 1; }
cat $O/ablz.log
