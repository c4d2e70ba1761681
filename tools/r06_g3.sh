# round 6 call 3: in-tree check (bench bit-exact + LZ4/snappy parity and stress tests), LZ4 parse A/B of the
# three batch-chain changes, the occupancy sweep (LDS padding), snappy A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_c; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/benchq.json 2> $O/benchq.err || { tail $O/benchq.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/benchq.json'));print('bench', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 bash tools/ab.sh e_none base e_dpp e_rest e_early > $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
cat $O/ab.log
AB_ROUNDS=1 AB_CORPORA=text timeout -k 10 200 bash tools/ab.sh base occ8 occ7 occ6 occ5 occ4 > $O/occ.log 2>&1 || { tail $O/occ.log; exit 1; }
cat $O/occ.log
PROF_ARGS="--codec snappy" AB_CORPORA="json mixed" timeout -k 10 300 bash tools/ab.sh sn_none sn_nearly base > $O/sn.log 2>&1 || { tail $O/sn.log; exit 1; }
cat $O/sn.log
