# round 6 call 14: LZ4 run batches take their lane mask and first position per branch (no ballot of a merged bool,
# no readlane); snappy loop state as ints: bench lines bit-exact, parity + stress tests, A/B against the head
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_n; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/bench_north.json 2> $O/bench_north.err || { tail $O/bench_north.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_north.json'));print('north', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --codec snappy --corpus json > $O/bench_snjson.json 2> $O/bench_snjson.err || { tail $O/bench_snjson.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_snjson.json'));print('snappy json', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --codec snappy --corpus mixed --chunk-kib 256 > $O/bench_snmixed.json 2> $O/bench_snmixed.err || { tail $O/bench_snmixed.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_snmixed.json'));print('snappy mixed b256', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_CORPORA="text json" AB_ROUNDS=3 timeout -k 10 400 bash tools/ab.sh head base > $O/ablz.log 2>&1 || { tail $O/ablz.log; exit 1; }
cat $O/ablz.log
PROF_ARGS="--codec snappy" AB_CORPORA="json mixed" AB_ROUNDS=3 timeout -k 10 500 bash tools/ab.sh head base > $O/absn.log 2>&1 || { tail $O/absn.log; exit 1; }
cat $O/absn.log
