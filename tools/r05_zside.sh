# zstd decode: the sequence kernel on a side stream -- zstd GPU tests (every path), then the A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05_zside}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 300 python3 tools/zside_ab.py > $O/ab.log 2>&1 || { tail -n 20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
