#!/bin/bash
# tools/r05_lnr.sh -- LZ4 parse kernel without the LDS input ring (table only: 16 KiB, 10 waves per CU
# instead of 9; P sides from memory), build/exp/lnr, against the in-tree library: A/B, bit-exactness
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_lnr; mkdir -p $O
for r in 1 2; do
  for v in base lnr; do
    if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    for cfg in "text 1024" "json 1024" "text 256"; do
      set -- $cfg
      echo -n "r$r $v lz4 $1 $2 MiB: "; LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --codec lz4 --mib $2 --reps 5 --corpus $1 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done 2>&1 | tee $O/ab.log
LZH_LIB=build/exp/lnr/liblzbench_hip.so timeout -k 10 300 python bench.py --no-e2e --no-cpu-baseline > $O/bench_lnr.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_lnr.json'));print('lnr north star', d['value'], 'bit_exact', d['bit_exact'], d['stage_ms'])"
