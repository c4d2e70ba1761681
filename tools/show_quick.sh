#!/bin/bash
# summary of tools/gpu_quick.sh outputs
tail -1 gpurun_out/quick.log; grep MISMATCH gpurun_out/quick.log | head -5
python3 -c "import json; d=json.load(open('gpurun_out/bench_lz4.json')); print(d['value'], d['stage_ms'], d['ratio_pct'])"
grep -v amdgpu.ids gpurun_out/stats.log
