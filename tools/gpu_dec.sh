#!/bin/bash
# tools/gpu_dec.sh TAG [VARIANT...] -- decoder iteration: bit-exact check, then kernel-only decode time
# (lz4 -b64 1 GiB text/json, snappy -b256 1 GiB mixed) for the in-tree build and each experiment build
tag=${1:-dec}; shift; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python tools/quick_gpu.py > $out/quick.log 2>&1 || { tail -5 $out/quick.log; exit 1; }
grep -q "BAD 0" $out/quick.log || { grep -v amdgpu.ids $out/quick.log | head -20; exit 1; }
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=build/exp/$v/liblzbench_hip.so; fi
  for c in text json; do
    echo -n "$v lz4 $c: "; LZH_LIB=$lib timeout -k 10 120 python tools/prof_kernels.py --mib 1024 --reps 3 --corpus $c --decompress 2>&1 | grep -v amdgpu.ids | tail -1
  done
  echo -n "$v snappy mixed -b256: "; LZH_LIB=$lib timeout -k 10 120 python tools/prof_kernels.py --codec snappy --chunk-kib 256 --mib 1024 --reps 3 --corpus mixed --decompress 2>&1 | grep -v amdgpu.ids | tail -1
done
echo "quick: $(tail -1 $out/quick.log)"
