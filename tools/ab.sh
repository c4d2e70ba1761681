#!/bin/bash
# tools/ab.sh VARIANT... -- A/B kernel-only compress timing of experiment builds on the same box,
# interleaved, AB_ROUNDS rounds (default 2) over AB_CORPORA (default "text json"), 1 GiB each;
# VARIANT "base" = the in-tree library (PROF_ARGS adds tools/prof_kernels.py options)
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    for c in ${AB_CORPORA:-text json}; do
      echo -n "r$r $v $c: "; LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --mib 1024 --reps 5 --corpus $c ${PROF_ARGS} 2>&1 | grep -v amdgpu.ids | tail -1
    done
  done
done
