#!/bin/bash
# tools/traffic_all.sh -- per-workload HBM traffic (rocprofv3 FETCH_SIZE / WRITE_SIZE, separate passes) for the
# bench line and every config line, each tagged with the code hash of every kernel it measured
# (tools/traffic_summary.py); output gpurun_out/${TRAFFIC_TAG:-traffic}/<workload>/traffic.json, to be copied to
# profiles/traffic_<workload>.json (bench.py traffic_for reads those only for the same machine code)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TRAFFIC_TAG:-traffic}
bash tools/pmc_traffic.sh $O/north lz4 text 64 1 1024 > /dev/null && \
bash tools/pmc_traffic.sh $O/c2 lz4 text 64 1 256 > /dev/null && \
bash tools/pmc_traffic.sh $O/c3 snappy mixed 256 1 1024 > /dev/null && \
bash tools/pmc_traffic.sh $O/c4lz4 lz4 json 64 1 1024 > /dev/null && \
bash tools/pmc_traffic.sh $O/c4sn snappy json 64 1 1024 > /dev/null && \
bash tools/pmc_traffic.sh $O/c5half zstd mixed 128 1 512 > /dev/null && \
bash tools/pmc_traffic.sh $O/c5 zstd mixed 128 1 1024 > /dev/null && \
bash tools/pmc_traffic.sh $O/fast3 lz4fast text 64 3 1024 > /dev/null && echo traffic done
