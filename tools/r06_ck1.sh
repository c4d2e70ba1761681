# round 6 checkpoint 1: the whole -m gpu suite, the default bench line (CPU baseline, e2e), its rocprofv3 kernel
# trace + stats, the one-GPU world-2 rehearsal (tools/gpu_round.sh steps)
set -o pipefail
cd $GRAFT_REPO_ROOT
LZH_TAG=${CK_TAG:-r06_ck} timeout -k 10 1100 bash tools/gpu_round.sh tests: bench prof ddp2
