# tools/r06_ab.sh TAG VARIANT... -- LZ4 parse A/B of experiment builds (tools/ab.sh, 1 GiB text and json, two
# interleaved rounds) into gpurun_out/TAG/ab.log; with CHECK=1 first the in-tree library's bench line
# (bit-exact against the reference digest) and the LZ4 GPU parity / stress tests
set -o pipefail
cd $GRAFT_REPO_ROOT
T=$1; shift
O=gpurun_out/$T; mkdir -p $O
if [ "$CHECK" = 1 ]; then
  timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/benchq.json 2> $O/benchq.err || { tail $O/benchq.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/benchq.json'));print('bench', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py ${TESTS} > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
timeout -k 10 900 bash tools/ab.sh "$@" > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
cat $O/ab.log
