#!/bin/bash
# tools/pmc_inst.sh OUTDIR VARIANT... -- instruction-mix counters (one pass) of the compress kernel for
# each experiment build (VARIANT "base" = the in-tree library), 1 GiB text
out=$1; shift
mkdir -p "$GRAFT_REPO_ROOT/$out"
for v in "$@"; do
  (
    if [ "$v" != base ]; then export LZH_LIB="$GRAFT_REPO_ROOT/build/exp/$v/liblzbench_hip.so"; fi
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVE_CYCLES --output-format csv -d "$GRAFT_REPO_ROOT/$out/$v/p0" -o pmc -- python3 "$GRAFT_REPO_ROOT/tools/prof_kernels.py" --mib 1024 --reps 1
  ) > "$GRAFT_REPO_ROOT/$out/$v.log" 2>&1 || { echo "$v failed"; tail -5 "$GRAFT_REPO_ROOT/$out/$v.log"; exit 1; }
  echo "== $v"; python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$GRAFT_REPO_ROOT/$out/$v" | grep -A8 "compress_v2"
done
