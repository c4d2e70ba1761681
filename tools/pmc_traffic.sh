#!/bin/bash
# tools/pmc_traffic.sh OUTDIR -- HBM-side traffic of the bench's kernels (1 GiB text, lz4 -b64):
# FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes (MI355X_MICROARCH.md, HBM section),
# compress kernel and decompress kernel runs; then tools/traffic_summary.py writes OUTDIR/traffic.json
out=$1; shift
mkdir -p "$GRAFT_REPO_ROOT/$out"
for mode in comp dec; do
  args="--mib 1024 --reps 1"; [ $mode = dec ] && args="$args --decompress"
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --pmc $c --output-format csv \
      -d "$GRAFT_REPO_ROOT/$out/$mode-$c" -o pmc -- python3 "$GRAFT_REPO_ROOT/tools/prof_kernels.py" $args) \
      > "$GRAFT_REPO_ROOT/$out/$mode-$c.log" 2>&1 || { echo "$mode $c failed"; tail -5 "$GRAFT_REPO_ROOT/$out/$mode-$c.log"; exit 1; }
  done
done
python3 "$GRAFT_REPO_ROOT/tools/traffic_summary.py" "$GRAFT_REPO_ROOT/$out"
