# tools/gpu_suite.sh OUT -- the whole -m gpu suite (one process, per-test timeout), log under gpurun_out/OUT
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-suite}; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?
tail -15 $O/pytest.log
exit $rc
