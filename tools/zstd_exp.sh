timeout -k 10 400 python -u -m pytest tests/test_gpu_zstd.py tests/test_gpu_zstd_compress.py -x -q --timeout 120 --timeout-method thread > gpurun_out/zq.log 2>&1; tail -2 gpurun_out/zq.log
bash tools/zstd_ab.sh base zprev
for r in 1 2; do for v in base zl0; do if [ $v = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi; for c in mixed text; do echo -n "c$r $v $c: "; LZH_LIB=$L timeout -k 10 200 python tools/prof_kernels.py --codec zstd --level 1 --chunk-kib 128 --corpus $c --mib 1024 --reps 2 2>&1 | grep -v amdgpu.ids | tail -1; done; done; done
