#!/bin/bash
# tools/gpu_iter.sh TAG -- one kernel iteration on the GPU box: bit-exact check on 4 corpora x 5 codec
# configs, LZ4 event counters + phase clocks, kernel-only compress/decompress time on 1 GiB text.
tag=${1:-iter}; out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 300 python tools/quick_gpu.py > $out/quick.log 2>&1 || { tail -5 $out/quick.log; exit 1; }
grep -q "BAD 0" $out/quick.log || { grep -v amdgpu.ids $out/quick.log | head -20; exit 1; }
timeout -k 10 200 python tools/lz4_stats.py text json > $out/stats.log 2>&1 || exit 1
for c in text json; do
  timeout -k 10 120 python tools/prof_kernels.py --mib 1024 --reps 3 --corpus $c > $out/comp_$c.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/prof_kernels.py --mib 1024 --reps 3 --decompress > $out/dec_text.log 2>&1 || exit 1
grep -hv amdgpu.ids $out/stats.log $out/comp_*.log $out/dec_*.log
echo "quick: $(tail -1 $out/quick.log)"
