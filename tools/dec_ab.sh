#!/bin/bash
# tools/dec_ab.sh VARIANT... -- decoder A/B: lz4 -b64 text, snappy -b256 mixed, zstd -b128 text
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    a=$(LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --mib 1024 --reps 5 --decompress 2>&1 | grep -v amdgpu.ids | tail -1)
    b=$(LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --codec snappy --chunk-kib 256 --corpus mixed --mib 1024 --reps 5 --decompress 2>&1 | grep -v amdgpu.ids | tail -1)
    c=$(LZH_LIB=$L timeout -k 10 120 python tools/zstd_prof.py --reps 3 2>&1 | grep -v amdgpu.ids | tail -1)
    echo "r$r $v | $a | $b | $c"
  done
done
