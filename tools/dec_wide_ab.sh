#!/bin/bash
# tools/dec_wide_ab.sh VARIANT... -- decoder A/B over chunk sizes (the output window choice depends on
# the chunk count): lz4 text -b64 / -b256, snappy mixed -b64 / -b256 / -b1024; "base" = in-tree
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    line="r$r $v"
    for cfg in "lz4 text 64" "lz4 text 256" "snappy mixed 64" "snappy mixed 256" "snappy mixed 1024"; do
      read -r co cp ck <<< "$cfg"
      t=$(LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --codec $co --corpus $cp --chunk-kib $ck --mib 1024 --reps 5 --decompress 2>&1 | grep -v amdgpu.ids | tail -1 | sed 's/.*: \([0-9.]*\) ms.*/\1/')
      line="$line | $co $cp -b$ck $t"
    done
    echo "$line"
  done
done
