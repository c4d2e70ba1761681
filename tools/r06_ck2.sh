# round 6 checkpoint 2: the config sweep and the per-workload PMC traffic (kernel-hash tagged)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${CK_TAG:-r06_ck}
mkdir -p gpurun_out/$T
timeout -k 10 600 bash tools/config_sweep.sh gpurun_out/$T/configs > gpurun_out/$T/sweep.log 2>&1 || { tail gpurun_out/$T/sweep.log; exit 1; }
cat gpurun_out/$T/sweep.log
TRAFFIC_TAG=$T/traffic timeout -k 10 500 bash tools/traffic_all.sh > gpurun_out/$T/traffic.log 2>&1 || { tail gpurun_out/$T/traffic.log; exit 1; }
tail -2 gpurun_out/$T/traffic.log
