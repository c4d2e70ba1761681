#!/bin/bash
# tools/stage_ab.sh VARIANT... -- bench stage times (parse / emit / scan+pack / decode) per variant, 2 rounds
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    echo -n "r$r $v: "
    LZH_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 5 --warmup 2 ${BENCH_ARGS} 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['stage_ms'], d.get('bit_exact'))"
  done
done
