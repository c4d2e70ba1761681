# per-workload HBM traffic (rocprofv3 FETCH_SIZE / WRITE_SIZE, separate passes) for every config line
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_traffic
bash tools/pmc_traffic.sh $O/c2 lz4 text 64 1 256 > /dev/null && \
bash tools/pmc_traffic.sh $O/c3 snappy mixed 256 1 1024 > /dev/null && \
bash tools/pmc_traffic.sh $O/c4lz4 lz4 json 64 1 1024 > /dev/null && \
bash tools/pmc_traffic.sh $O/c4sn snappy json 64 1 1024 > /dev/null && \
bash tools/pmc_traffic.sh $O/c5half zstd mixed 128 1 512 > /dev/null && \
bash tools/pmc_traffic.sh $O/fast3 lz4fast text 64 3 1024 > /dev/null && echo traffic done
