set -o pipefail
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "lz4fast" > gpurun_out/fast_t.log 2>&1 || { tail -30 gpurun_out/fast_t.log; exit 1; }
tail -3 gpurun_out/fast_t.log
for v in old base; do
  if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
  for a in 1 3 17; do
    c=lz4fast; [ $a = 1 ] && c=lz4
    LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --codec $c --level $a --mib 1024 --reps 3 2>&1 | grep -v amdgpu.ids | tail -1
  done
done
