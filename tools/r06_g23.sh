# round 6 call 23: snappy parse -- the loop state runm (snA) and runm / retest / U (base) without the batch-head readfirstlanes:
# snappy bench lines bit-exact, snappy parity / stress, A/B against the head
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_x; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --codec snappy --corpus json > $O/bench_snjson.json 2> $O/bench_snjson.err || { tail $O/bench_snjson.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_snjson.json'));print('snappy json', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --codec snappy --corpus mixed --chunk-kib 256 > $O/bench_snmixed.json 2> $O/bench_snmixed.err || { tail $O/bench_snmixed.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_snmixed.json'));print('snappy mixed b256', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py tests/test_gpu_rows.py -k snappy > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
PROF_ARGS="--codec snappy" AB_CORPORA="json mixed" AB_ROUNDS=3 timeout -k 10 600 bash tools/ab.sh head snA base > $O/absn.log 2>&1 || { tail $O/absn.log; exit 1; }
cat $O/absn.log
