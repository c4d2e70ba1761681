#!/bin/bash
# tools/pmc_icache.sh OUTDIR [prof_kernels args] -- instruction-fetch counters (I-cache hits /
# misses, fetch level) of the compress kernel on 1 GiB text, one pass
out=$1; shift
mkdir -p "$GRAFT_REPO_ROOT/$out"
G="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_IFETCH_LEVEL SQ_INSTS_VALU SQ_WAVE_CYCLES"
(
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d "$GRAFT_REPO_ROOT/$out/p0" -o pmc -- python3 "$GRAFT_REPO_ROOT/tools/prof_kernels.py" --mib 1024 --reps 1 "$@"
) > "$GRAFT_REPO_ROOT/$out/p0.log" 2>&1 || { echo "pmc failed"; tail -5 "$GRAFT_REPO_ROOT/$out/p0.log"; exit 1; }
python3 "$GRAFT_REPO_ROOT/tools/pmc_summary.py" "$GRAFT_REPO_ROOT/$out" | grep -A9 "compress_v2\|decompress_v2"
