#!/bin/bash
# tools/r05_zg.sh -- zstd match finder: no candidate gathers in collision-free batches (build/exp/zg)
# against the in-tree library (r05_zu head): A/B (compress stage, 1 GiB -b128), zstd compress tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_zg; mkdir -p $O
for r in 1 2; do
  for v in base zg; do
    if [ "$v" = base ]; then L=""; else L=build/exp/$v/liblzbench_hip.so; fi
    for c in mixed text; do
      echo -n "r$r $v zstd1 $c -b128: "; LZH_LIB=$L timeout -k 10 120 python tools/prof_kernels.py --codec zstd --level 1 --chunk-kib 128 --mib 1024 --reps 3 --corpus $c 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
    done
  done
done 2>&1 | tee $O/ab.log
LZH_LIB=build/exp/zg/liblzbench_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_zstd_compress.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
exit $rc
