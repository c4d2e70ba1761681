# round 6, call 2: zstd GPU tests after the seq-kernel bound / side-stream changes; zstd e2e A/B (round-5 head
# library vs this one: side streams per caller stream)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_b; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_zstd.py tests/test_gpu_zstd_compress.py tests/test_multi.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for v in r05head base; do
    if [ $v = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    LZH_LIB=$L timeout -k 10 300 python -u bench.py --codec zstd --chunk-kib 128 --corpus mixed --no-cpu-baseline --steps 3 --warmup 1 > $O/e2e_${v}_$r.json 2> $O/e2e_${v}_$r.err || { tail $O/e2e_${v}_$r.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open('$O/e2e_${v}_$r.json'));print('$v r$r', d['value'], d['ms_per_step'], d['bit_exact'], json.dumps(d.get('e2e')))"
  done
done
