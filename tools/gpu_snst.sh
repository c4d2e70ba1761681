timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "snappy" > gpurun_out/sn_t.log 2>&1; tail -2 gpurun_out/sn_t.log
for v in old base; do
  L=""; [ $v = old ] && L=build/exp/old/liblzbench_hip.so
  for a in "--codec snappy --chunk-kib 256 --corpus mixed" "--codec snappy --corpus text"; do
    echo -n "$v $a: "; LZH_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 $a 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms'])"
  done
done
