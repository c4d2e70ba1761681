# round 6 call 16: the LZ4 / snappy group decoders' far / done / overlap / read-round sets and chain_members' result
# as lane masks from single-compare ballots: bench lines bit-exact, the decode-side GPU suites, decoder A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_p; mkdir -p $O
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > $O/bench_north.json 2> $O/bench_north.err || { tail $O/bench_north.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_north.json'));print('north', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline --codec snappy --corpus mixed --chunk-kib 256 > $O/bench_snmixed.json 2> $O/bench_snmixed.err || { tail $O/bench_snmixed.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_snmixed.json'));print('snappy mixed b256', d['value'], d['stage_ms'], 'bit_exact', d['bit_exact'])"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py tests/test_gpu_fuzz.py tests/test_gpu_windows.py tests/test_gpu_frames.py tests/test_gpu_snappy_split.py tests/test_gpu_rows.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 bash tools/dec_ab.sh head base > $O/abdec.log 2>&1 || { tail $O/abdec.log; exit 1; }
cat $O/abdec.log
for r in 1 2; do for v in head base; do if [ $v = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
  echo "r$r $v json: $(LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --mib 1024 --reps 5 --decompress --corpus json 2>&1 | grep -v amdgpu.ids | tail -1)"; done; done >> $O/abdec.log
tail -4 $O/abdec.log
