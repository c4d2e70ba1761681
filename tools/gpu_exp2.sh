mkdir -p gpurun_out/exp2
for v in "$@"; do
  for c in text json; do
    echo -n "$v $c: "; LZH_LIB=build/exp/$v/liblzbench_hip.so timeout -k 10 120 python tools/prof_kernels.py --mib 1024 --reps 3 --corpus $c 2>&1 | grep -v amdgpu.ids | tail -1
  done
done
