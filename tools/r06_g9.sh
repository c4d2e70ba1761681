# round 6 call 9: LZ4 parse ballot / window-logic cuts and the zstd match finder's single-compare ballots: benches
# bit-exact (north star, zstd-1 mixed -b128), LZ4 parity / stress and zstd compress tests, A/B against the head
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_i; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/benchq.json 2> $O/benchq.err || { tail $O/benchq.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/benchq.json'));print('bench', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --codec zstd --chunk-kib 128 --corpus mixed > $O/bench_zstd.json 2> $O/bench_zstd.err || { tail $O/bench_zstd.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_zstd.json'));print('zstd', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 800 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py tests/test_gpu_zstd_compress.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_ROUNDS=3 timeout -k 10 400 bash tools/ab.sh head base > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
cat $O/ab.log
PROF_ARGS="--codec zstd --chunk-kib 128" AB_CORPORA="mixed text" timeout -k 10 400 bash tools/ab.sh head base > $O/abz.log 2>&1 || { tail $O/abz.log; exit 1; }
cat $O/abz.log
