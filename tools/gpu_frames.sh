#!/bin/bash
# tools/gpu_frames.sh TAG -- framed-format GPU tests, the LZ4 parity tests, a short bench (regression check)
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_parity.py tests/test_driver.py -x -v --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 \
&& timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > $out/bench.json 2> $out/bench.err
rc=$?
echo "rc=$rc"; grep -E "passed|failed|FAILED|Error" $out/pytest.log | tail -8; cat $out/bench.json
exit $rc
