#!/bin/bash
# tools/pmc_sq.sh OUTDIR <prof_kernels.py args...>
# instruction-mix / wait / cache counters of the codec kernels, one rocprofv3 --pmc pass per group
set -o pipefail
out=$1; shift
cd "$GRAFT_REPO_ROOT"
groups=(
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH"
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES"
  "TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT"
  "FETCH_SIZE"
  "WRITE_SIZE"
)
mkdir -p "$out"
i=0
for g in "${groups[@]}"; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --pmc $g --output-format csv -d "$GRAFT_REPO_ROOT/$out/p$i" -o pmc -- python3 "$GRAFT_REPO_ROOT/tools/prof_kernels.py" "$@") > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -20 "$out/p$i.log"; exit 1; }
  i=$((i+1))
done
echo done
