#!/bin/bash
# tools/config_sweep.sh OUTDIR -- one bench line per BASELINE.json config that fits one GPU
# (configs 4 and 5 at their per-GPU shares of 8 GPUs, plus 1 GiB), and lz4fast,3.
out=${1:-gpurun_out/sweep}; mkdir -p $out
set -o pipefail
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -3 $out/$name.err; return 1; }; echo "$name: $(python3 -c "import json;d=json.load(open('$out/$name.json'));print(d['value'], d['unit'], 'ratio', d['ratio_pct'], 'comp', d['comp_MBps'], 'decomp', d['decomp_MBps'], 'bit_exact', d.get('bit_exact'), 'cpu1', (d['cpu_baseline'] or {}).get('value'), 'cpuN', (d.get('cpu_baseline_all_cores') or {}).get('value'))")"; }
run north_lz4_b64_text1g && \
run c2_lz4_b64_text256 --size-mib 256 && \
run c3_snappy_b256_mixed1g --codec snappy --chunk-kib 256 --corpus mixed && \
run c4_lz4_b64_json1g --corpus json && \
run c4_snappy_b64_json1g --codec snappy --corpus json && \
run c5_zstd1_b128_mixed512 --codec zstd --level 1 --chunk-kib 128 --corpus mixed --size-mib 512 && \
run c5_zstd1_b128_mixed1g --codec zstd --level 1 --chunk-kib 128 --corpus mixed && \
run lz4fast3_b64_text1g --codec lz4fast --level 3
