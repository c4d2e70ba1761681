#!/bin/bash
# tools/gpu_zstd.sh TAG -- zstd compression check on the GPU box: the -m gpu zstd tests, then the
# zstd -b128 bench line on 1 GiB mixed.  Output in gpurun_out/TAG/.
tag=${1:-zstd}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd_compress.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest_zstd.log 2>&1
rc=$?
tail -15 $out/pytest_zstd.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --codec zstd --chunk-kib 128 --corpus mixed --steps 3 --warmup 1 > $out/bench_zstd.json 2> $out/bench_zstd.err
rc=$?
cat $out/bench_zstd.json; tail -3 $out/bench_zstd.err
exit $rc
