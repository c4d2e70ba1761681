#!/bin/bash
# tools/r05_zfinal.sh -- the in-tree library after the zstd match-finder changes: zstd GPU tests, config 5 at the
# 512 MiB share and 1 GiB (bit-exact against the reference digests), and the north-star bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_zfinal; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_zstd_compress.py tests/test_gpu_zstd.py > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/config_sweep.sh $O/configs > $O/sweep.log 2>&1 || { tail $O/sweep.log; exit 1; }
cat $O/sweep.log
