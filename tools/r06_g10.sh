# round 6 call 10: decoder groups' uniform fast bound check (LZH_DEC_FASTCHK) and the zstd match finder's single-
# compare ballots: decoder tests (parity, fuzz verdicts, windows, snappy split), bench lines bit-exact, A/B vs head
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_j; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/benchq.json 2> $O/benchq.err || { tail $O/benchq.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/benchq.json'));print('bench', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --codec snappy --chunk-kib 256 --corpus mixed > $O/bench_sn.json 2> $O/bench_sn.err || { tail $O/bench_sn.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_sn.json'));print('snappy', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_windows.py tests/test_gpu_snappy_split.py tests/test_gpu_frames.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
PROF_ARGS="--decompress" AB_ROUNDS=3 timeout -k 10 400 bash tools/ab.sh head base > $O/abdec.log 2>&1 || { tail $O/abdec.log; exit 1; }
cat $O/abdec.log
PROF_ARGS="--decompress --codec snappy --chunk-kib 256" AB_CORPORA=mixed timeout -k 10 300 bash tools/ab.sh head base > $O/abdecsn.log 2>&1 || { tail $O/abdecsn.log; exit 1; }
cat $O/abdecsn.log
PROF_ARGS="--codec zstd --level 1 --chunk-kib 128" AB_CORPORA="mixed text" timeout -k 10 400 bash tools/ab.sh head base > $O/abz.log 2>&1 || { tail $O/abz.log; exit 1; }
cat $O/abz.log
