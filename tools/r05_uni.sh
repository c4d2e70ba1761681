#!/bin/bash
# tools/r05_uni.sh -- uniform batch-loop state in the LZ4 / snappy parse kernels: A/B against the head
# library (build/exp/h0) on one box (compress stage, 1 GiB, 5 reps, 2 rounds), then the instruction
# mix of both (tools/pmc_inst.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_uni; mkdir -p $O
for r in 1 2; do
  for v in h0 base; do
    if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    for cfg in "lz4 text" "lz4 json" "snappy json"; do
      set -- $cfg
      echo -n "r$r $v $1 $2: "; LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --codec $1 --mib 1024 --reps 5 --corpus $2 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done 2>&1 | tee $O/ab.log
bash tools/pmc_inst.sh gpurun_out/r05_uni/pmc h0 base 2>&1 | tee $O/pmc.log
