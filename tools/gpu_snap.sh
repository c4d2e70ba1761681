#!/bin/bash
# tools/gpu_snap.sh -- snappy parity suites + compress timing (old = build/exp/old, base = in-tree)
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_stress.py tests/test_gpu_rows.py -k "snappy" > gpurun_out/snap_t.log 2>&1 || { tail -30 gpurun_out/snap_t.log; exit 1; }
tail -2 gpurun_out/snap_t.log
for v in ${SNAP_VARIANTS:-old base}; do
  if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
  LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --codec snappy --chunk-kib 256 --corpus mixed --mib 1024 --reps 3 2>&1 | grep -v amdgpu.ids | tail -1
  LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --codec snappy --chunk-kib 64 --corpus text --mib 1024 --reps 3 2>&1 | grep -v amdgpu.ids | tail -1
  LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --codec snappy --chunk-kib 64 --corpus json --mib 1024 --reps 3 2>&1 | grep -v amdgpu.ids | tail -1
done
