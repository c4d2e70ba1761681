#!/bin/bash
# tools/zstdc_ab.sh VARIANT... -- zstd-1 -b128 compression kernel A/B (1 GiB mixed and text); "base" = in-tree
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    for c in mixed text; do
      echo -n "r$r $v $c: "; LZH_LIB=$L timeout -k 10 200 python tools/prof_kernels.py --codec zstd --level 1 --chunk-kib 128 --corpus $c --mib 1024 --reps 3 2>&1 | grep -v amdgpu.ids | tail -1
    done
  done
done
