#!/bin/bash
# tools/gpu_snap.sh TAG [VARIANT...] -- snappy compressor iteration: bit-exact check (4 corpora x 5 configs),
# then kernel-only snappy compress time (-b256 mixed, -b64 text) for the in-tree build and experiment builds
tag=${1:-snap}; shift; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python tools/quick_gpu.py > $out/quick.log 2>&1 || { tail -5 $out/quick.log; exit 1; }
grep -q "BAD 0" $out/quick.log || { grep -v amdgpu.ids $out/quick.log | head -20; exit 1; }
for v in base "$@"; do
  if [ "$v" = base ]; then lib=""; else lib=build/exp/$v/liblzbench_hip.so; fi
  echo -n "$v snappy mixed -b256: "; LZH_LIB=$lib timeout -k 10 120 python tools/prof_kernels.py --codec snappy --chunk-kib 256 --mib 1024 --reps 3 --corpus mixed 2>&1 | grep -v amdgpu.ids | tail -1
  echo -n "$v snappy text -b64: "; LZH_LIB=$lib timeout -k 10 120 python tools/prof_kernels.py --codec snappy --chunk-kib 64 --mib 1024 --reps 3 --corpus text 2>&1 | grep -v amdgpu.ids | tail -1
done
echo "quick: $(tail -1 $out/quick.log)"
