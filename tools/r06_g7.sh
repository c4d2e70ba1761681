# round 6 call 7: LZ4 parse instruction cuts (slot groups from LDS masks, a 5-instruction walk step, the probed /
# inserted sets as lane masks): bench bit-exact, LZ4 parity / stress tests, A/B against the previous head and with
# each cut off (nogrp / nowalk / nomask)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_g; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/benchq.json 2> $O/benchq.err || { tail $O/benchq.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/benchq.json'));print('bench', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --corpus json > $O/bench_json.json 2> $O/bench_json.err || { tail $O/bench_json.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_json.json'));print('lz4 json', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 bash tools/ab.sh head base nogrp nowalk nomask > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
cat $O/ab.log
