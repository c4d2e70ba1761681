# zstd compress: single-block frames split over the side stream -- compress parity tests, then the A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05_zsplitc}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd_compress.py tests/test_zstd_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 300 python3 tools/zsplitc_ab.py > $O/ab.log 2>&1 || { tail -n 20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
