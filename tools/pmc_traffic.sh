#!/bin/bash
# tools/pmc_traffic.sh OUTDIR [CODEC CORPUS CHUNK_KIB LEVEL MIB] -- HBM-side traffic of the bench's kernels
# (default: 1 GiB text, lz4 -b64): FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes
# (MI355X_MICROARCH.md, HBM section), compress kernel and decompress kernel runs; then
# tools/traffic_summary.py writes OUTDIR/traffic.json keyed by bench.py's workload key
out=$1; shift
codec=${1:-lz4}; corpus=${2:-text}; ck=${3:-64}; lvl=${4:-1}; mib=${5:-1024}
mkdir -p "$GRAFT_REPO_ROOT/$out"
for mode in comp dec; do
  args="--mib $mib --reps 1 --codec $codec --corpus $corpus --chunk-kib $ck --level $lvl"; [ $mode = dec ] && args="$args --decompress"
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --pmc $c --output-format csv \
      -d "$GRAFT_REPO_ROOT/$out/$mode-$c" -o pmc -- python3 "$GRAFT_REPO_ROOT/tools/prof_kernels.py" $args) \
      > "$GRAFT_REPO_ROOT/$out/$mode-$c.log" 2>&1 || { echo "$mode $c failed"; tail -5 "$GRAFT_REPO_ROOT/$out/$mode-$c.log"; exit 1; }
  done
done
python3 "$GRAFT_REPO_ROOT/tools/traffic_summary.py" "$GRAFT_REPO_ROOT/$out" "$codec/$lvl/$ck/$corpus/$((mib << 20))"
