#!/bin/bash
# tools/pmc_parse.sh OUTDIR [VARIANT...] -- per-class instruction and stall counters of the compress kernels
# (three rocprofv3 --pmc passes, kernel trace only), 1 GiB text (PROF_ARGS adds tools/prof_kernels.py options);
# VARIANT "base" = the in-tree library, else build/exp/VARIANT (tools/exp_build.sh)
out=$1; shift
[ $# -eq 0 ] && set -- base
mkdir -p "$GRAFT_REPO_ROOT/$out"
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES"
G2="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INST_CYCLES_SALU"
G3="SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SENDMSG SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_BUSY_CYCLES SQ_WAVES"
for v in "$@"; do
  i=0
  for g in "$G1" "$G2" "$G3"; do
  (
    if [ "$v" != base ]; then export LZH_LIB="$GRAFT_REPO_ROOT/build/exp/$v/liblzbench_hip.so"; fi
    cd /tmp && export TMPDIR=/tmp
    timeout -s KILL 90 rocprofv3 --pmc $g --output-format csv -d "$GRAFT_REPO_ROOT/$out/$v/p$i" -o pmc -- python3 "$GRAFT_REPO_ROOT/tools/prof_kernels.py" --mib 1024 --reps 1 ${PROF_ARGS}
  ) > "$GRAFT_REPO_ROOT/$out/$v.p$i.log" 2>&1 || { echo "$v pass $i failed"; tail -5 "$GRAFT_REPO_ROOT/$out/$v.p$i.log"; exit 1; }
  i=$((i+1))
  done
  echo "== $v"; python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$GRAFT_REPO_ROOT/$out/$v" | grep -A24 "parse_kernel"
done
