# round 6 call 6: window loads issued after the candidate loads (compiler-tracked waits) in both parse kernels:
# benches bit-exact, parity / stress tests, A/B: LZ4 v2 (in-tree) vs v1 (rwv1: window load at the batch top);
# snappy register window v2 (in-tree, 5 waves per CU) vs the ring kernel (snrw0)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_f; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/benchq.json 2> $O/benchq.err || { tail $O/benchq.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/benchq.json'));print('bench', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --codec snappy --corpus json > $O/bench_snjson.json 2> $O/bench_snjson.err || { tail $O/bench_snjson.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_snjson.json'));print('snappy json', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --codec snappy --corpus mixed --chunk-kib 256 > $O/bench_snmixed.json 2> $O/bench_snmixed.err || { tail $O/bench_snmixed.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_snmixed.json'));print('snappy mixed b256', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 bash tools/ab.sh rwv1 base > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
cat $O/ab.log
PROF_ARGS="--codec snappy" AB_CORPORA="json mixed" timeout -k 10 300 bash tools/ab.sh snrw0 base > $O/absn.log 2>&1 || { tail $O/absn.log; exit 1; }
cat $O/absn.log
