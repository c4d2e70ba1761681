set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_g; mkdir -p $O
timeout -k 10 300 python tools/rows_diff.py zstd 128 4096 mixed 1 8 > $O/rows_zstd.log 2>&1; rc=$?; cat $O/rows_zstd.log | grep -v amdgpu.ids
exit $rc
