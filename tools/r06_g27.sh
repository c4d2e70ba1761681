# round 6 call 27: the LZ4 file under max-memory-clause (in-tree now): north-star line bit-exact, LZ4 parity / stress /
# rows / frames; the snappy file under max-ilp (snilp) / the default (sndef), the decoders under the default (decdef) /
# max-memory-clause (decmmc): A/B against the head
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_zb; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/bench_north.json 2> $O/bench_north.err || { tail $O/bench_north.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_north.json'));print('north', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py tests/test_gpu_rows.py tests/test_gpu_frames.py -k "lz4 or LZ4" > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
PROF_ARGS="--codec snappy" AB_CORPORA="json mixed" AB_ROUNDS=2 timeout -k 10 600 bash tools/ab.sh head snilp sndef > $O/absn.log 2>&1 || { tail $O/absn.log; exit 1; }
cat $O/absn.log
timeout -k 10 600 bash tools/dec_ab.sh head decdef decmmc > $O/abdec.log 2>&1 || { tail $O/abdec.log; exit 1; }
cat $O/abdec.log
