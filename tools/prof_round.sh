#!/bin/bash
# tools/prof_round.sh TAG [bench args...] -- rocprofv3 kernel trace + stats of one bench run
# (no CPU baseline / e2e legs); summary in gpurun_out/TAG/prof/run_kernel_stats.csv
tag=$1; shift
out=$GRAFT_REPO_ROOT/gpurun_out/$tag
mkdir -p $out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-e2e --steps 3 --warmup 1 "$@" > $out/bench.json 2> $out/bench.err
rc=$?
cat $out/bench.json
python3 - "$out/prof" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:60]:60s} calls {r['Calls']:>5s} avg_ms {float(r['AverageNs'])/1e6:9.3f} pct {float(r['Percentage']):6.2f}")
PY
exit $rc
