#!/bin/bash
# tools/pmc_zstd.sh OUTDIR -- instruction mix of the zstd decode kernel (two passes)
out=$1; shift
mkdir -p "$GRAFT_REPO_ROOT/$out"
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES"
G2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INST_CYCLES_SALU"
i=0
for g in "$G1" "$G2"; do
  ( cd /tmp && export TMPDIR=/tmp
    timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d "$GRAFT_REPO_ROOT/$out/p$i" -o pmc -- python3 "$GRAFT_REPO_ROOT/tools/zstd_prof.py" --reps 1 "$@"
  ) > "$GRAFT_REPO_ROOT/$out/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$GRAFT_REPO_ROOT/$out/p$i.log"; exit 1; }
  i=$((i+1))
done
python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$GRAFT_REPO_ROOT/$out" | grep -A16 "zstd_decompress"
