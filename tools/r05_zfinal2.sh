#!/bin/bash
# tools/r05_zfinal2.sh -- the in-tree library after r05_zg: zstd GPU tests, config 5 (512 MiB share and 1 GiB,
# bit-exact against the reference digests) and the north-star bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05_zfinal2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_zstd_compress.py tests/test_gpu_zstd.py > $O/pytest.log 2>&1 || { tail -5 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for a in "c5_zstd1_b128_mixed512 --size-mib 512" "c5_zstd1_b128_mixed1g"; do
  set -- $a; n=$1; shift
  timeout -k 10 400 python bench.py --codec zstd --level 1 --chunk-kib 128 --corpus mixed "$@" > $O/$n.json 2> $O/$n.err || { tail -3 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], 'comp', d['comp_MBps'], 'decomp', d['decomp_MBps'], 'bit_exact', d['bit_exact'], d['stage_ms'])"
done
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -3 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('north', d['value'], 'bit_exact', d['bit_exact'], d['stage_ms'])"
