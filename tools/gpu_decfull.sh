#!/bin/bash
# tools/gpu_decfull.sh VARIANT... -- full GPU suite, then decoder A/B and decoder counters
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/dec_t.log 2>&1
rc=$?; tail -3 gpurun_out/dec_t.log; [ $rc -eq 0 ] || exit $rc
bash tools/dec_ab.sh "$@" || exit 1
if [ -f build/exp/decst/liblzbench_hip.so ]; then
  export LZH_LIB=build/exp/decst/liblzbench_hip.so
  timeout -k 10 200 python tools/dec_stats.py lz4 text 2>&1 | grep -v amdgpu.ids
  timeout -k 10 200 python tools/dec_stats.py lz4 json 2>&1 | grep -v amdgpu.ids
fi
