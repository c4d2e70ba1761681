set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06_a
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/r06_a/avail.txt 2>&1 || true
cd $GRAFT_REPO_ROOT
grep -o "SQ_[A-Z_0-9]*" gpurun_out/r06_a/avail.txt | sort -u > gpurun_out/r06_a/sq_counters.txt || true
LZH_TAG=r06_a timeout -k 10 900 bash tools/gpu_round.sh benchq prof && \
timeout -k 10 120 python tools/lz4_stats.py text json > gpurun_out/r06_a/lz4_stats.txt 2>&1 && \
bash tools/pmc_parse.sh gpurun_out/r06_a/pmc base > gpurun_out/r06_a/pmc.log 2>&1; echo pmc rc=$?; tail -30 gpurun_out/r06_a/pmc.log
