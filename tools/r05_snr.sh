#!/bin/bash
# tools/r05_snr.sh -- snappy parse kernel without the LDS input ring (table only: 32 KiB, 5 waves per CU
# instead of 4; P sides from memory), build/exp/snr, against the in-tree library: A/B, bit-exactness
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_snr; mkdir -p $O
for r in 1 2; do
  for v in base snr; do
    if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    for cfg in "json 64" "mixed 256" "text 64"; do
      set -- $cfg
      echo -n "r$r $v snappy $1 -b$2: "; LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --codec snappy --mib 1024 --reps 5 --corpus $1 --chunk-kib $2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done 2>&1 | tee $O/ab.log
LZH_LIB=build/exp/snr/liblzbench_hip.so timeout -k 10 300 python bench.py --codec snappy --corpus json --no-e2e --no-cpu-baseline > $O/bench_snr_json.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_snr_json.json'));print('snr json -b64', d['value'], 'bit_exact', d['bit_exact'], d['stage_ms'])"
LZH_LIB=build/exp/snr/liblzbench_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stress.py -k snappy > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
exit $rc
