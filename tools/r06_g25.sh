# round 6 call 25: LZ4 parse -- the switch to stride batches at the next batch head (runb 2) and the run batch's state updates on one path:
# north-star line bit-exact, LZ4 parity / stress / rows / frames, A/B against the head
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_z; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/bench_north.json 2> $O/bench_north.err || { tail $O/bench_north.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_north.json'));print('north', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py tests/test_gpu_rows.py tests/test_gpu_frames.py -k "lz4 or LZ4" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_CORPORA="text json" AB_ROUNDS=3 timeout -k 10 500 bash tools/ab.sh head base > $O/ablz.log 2>&1 || { tail $O/ablz.log; exit 1; }
cat $O/ablz.log
