#!/bin/bash
# tools/gpu_tail.sh -- parse-kernel tail: kernel time vs chunk count around the wave-slot multiple
for m in 896 1008 1024 1152; do
  timeout -k 10 120 python tools/prof_kernels.py --mib $m --reps 5 2>&1 | grep -v amdgpu.ids | tail -1
done
timeout -k 10 120 python tools/prof_kernels.py --codec snappy --chunk-kib 256 --corpus mixed --mib 1024 --reps 3 2>&1 | grep -v amdgpu.ids | tail -1
timeout -k 10 120 python tools/prof_kernels.py --codec snappy --chunk-kib 64 --corpus text --mib 1024 --reps 3 2>&1 | grep -v amdgpu.ids | tail -1
