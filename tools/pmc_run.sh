#!/bin/bash
# tools/pmc_run.sh OUTDIR "<counters pass 1>" "<counters pass 2>" ... -- <program args>
# one rocprofv3 --pmc pass per counter group (kernel-trace only; no sys/runtime traces)
set -o pipefail
out=$1; shift
groups=()
while [ "$1" != "--" ]; do groups+=("$1"); shift; done
shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$out"
i=0
for g in "${groups[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $g --output-format csv -d "$out/p$i" -o pmc -- python3 "$@" > "$out/p$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
  i=$((i+1))
done
echo done
