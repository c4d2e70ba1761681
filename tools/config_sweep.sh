#!/bin/bash
# tools/config_sweep.sh OUTDIR -- one bench line per BASELINE.json config that fits one GPU
# (config 4 at its per-GPU share), plus the zstd decode side of config 5.
out=${1:-gpurun_out/sweep}; mkdir -p $out
set -o pipefail
run() { local name=$1; shift; timeout -k 10 400 python bench.py "$@" > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -3 $out/$name.err; return 1; }; echo "$name: $(python3 -c "import json;d=json.load(open('$out/$name.json'));print(d['value'], d['unit'], 'ratio', d['ratio_pct'], 'comp', d['comp_MBps'], 'decomp', d['decomp_MBps'], 'cpu1', (d['cpu_baseline'] or {}).get('value'))")"; }
run c2_lz4_b64_text256 --size-mib 256 && \
run c3_snappy_b256_mixed1g --codec snappy --chunk-kib 256 --corpus mixed && \
run c4_lz4_b64_json1g --corpus json && \
run c4_snappy_b64_json1g --codec snappy --corpus json && \
run lz4fast3_b64_text1g --codec lz4fast --level 3 && \
timeout -k 10 400 python tools/zstd_prof.py --mib 4096 --chunk 131072 --corpus mixed --reps 2 > $out/c5_zstd_decode_mixed4g.log 2>&1 && grep -v amdgpu.ids $out/c5_zstd_decode_mixed4g.log
