#!/bin/bash
# tools/exp_time.sh NAME... -- kernel-only compress time of each experiment build (1 GiB text)
for n in "$@"; do
  echo -n "$n: "
  LZH_LIB=build/exp/$n/liblzbench_hip.so timeout -k 10 120 python tools/prof_kernels.py --mib 1024 --reps 3 ${EXP_ARGS} 2>&1 | grep -v amdgpu.ids | tail -1
done
