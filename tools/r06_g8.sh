# round 6 call 8: LZ4 parse instruction cuts without the LDS slot-group masks: bench bit-exact, parity tests, A/B
# (3 rounds) against the previous head, with 9 waves per CU (p512), without the walk / mask cuts; decoder PMC
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_h; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/benchq.json 2> $O/benchq.err || { tail $O/benchq.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/benchq.json'));print('bench', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
AB_ROUNDS=3 timeout -k 10 700 bash tools/ab.sh head base p512 nowalk2 nomask2 > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
cat $O/ab.log
PROF_ARGS="--decompress" bash tools/pmc_parse.sh gpurun_out/r06_h/pmc_dec base > $O/pmc_dec.log 2>&1; echo pmc rc=$?
python3 tools/pmc_summary.py gpurun_out/r06_h/pmc_dec/base | grep -A24 "decompress_v2_kernel"
PROF_ARGS="--codec snappy" AB_CORPORA="json mixed" timeout -k 10 300 bash tools/ab.sh head base > $O/absn.log 2>&1 || { tail $O/absn.log; exit 1; }
cat $O/absn.log
