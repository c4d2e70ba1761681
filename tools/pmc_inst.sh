#!/bin/bash
# tools/pmc_inst.sh OUTDIR VARIANT... -- instruction-mix and stall counters (two passes) of the compress
# kernel for each experiment build (VARIANT "base" = the in-tree library), 1 GiB text
out=$1; shift
mkdir -p "$GRAFT_REPO_ROOT/$out"
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES"
G2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INST_CYCLES_SALU"
for v in "$@"; do
  i=0
  for g in "$G1" "$G2"; do
  (
    if [ "$v" != base ]; then export LZH_LIB="$GRAFT_REPO_ROOT/build/exp/$v/liblzbench_hip.so"; fi
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 120 rocprofv3 --pmc $g --output-format csv -d "$GRAFT_REPO_ROOT/$out/$v/p$i" -o pmc -- python3 "$GRAFT_REPO_ROOT/tools/prof_kernels.py" --mib 1024 --reps 1 ${PROF_ARGS}
  ) > "$GRAFT_REPO_ROOT/$out/$v.p$i.log" 2>&1 || { echo "$v failed"; tail -5 "$GRAFT_REPO_ROOT/$out/$v.p$i.log"; exit 1; }
  i=$((i+1))
  done
  echo "== $v"; python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$GRAFT_REPO_ROOT/$out/$v" | grep -A16 "_kernel"
done
