#!/bin/bash
# tools/zstd_ab.sh VARIANT... -- zstd decode A/B (text and mixed, 256 MiB, -b128); "base" = in-tree library
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    for c in text mixed; do
      echo -n "r$r $v: "; LZH_LIB=$L timeout -k 10 120 python tools/zstd_prof.py --corpus $c --mib 256 --reps 3 2>&1 | grep -v amdgpu.ids | tail -1
    done
  done
done
