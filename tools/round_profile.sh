#!/bin/bash
# tools/round_profile.sh TAG -- the artifacts of a round for profiles/: PMC traffic passes
# (FETCH_SIZE / WRITE_SIZE, separate runs), a rocprofv3 kernel-trace + stats run of the bench,
# and the full default bench line (CPU baseline, e2e).
set -o pipefail
tag=$1
out=gpurun_out/$tag
mkdir -p $out
bash tools/pmc_traffic.sh $out/traffic > $out/traffic.log 2>&1 || { echo "traffic failed"; tail -5 $out/traffic.log; exit 1; }
cp $out/traffic/traffic.json profiles/traffic_$(basename $out).json
LZH_TAG=$tag bash tools/gpu_round.sh prof > $out/rocprof.log 2>&1 || { echo "rocprof failed"; tail -5 $out/rocprof.log; exit 1; }
timeout -k 10 500 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
cat $out/bench.json
tail -12 $out/rocprof.log
