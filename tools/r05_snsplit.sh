# snappy fragment-parallel decode: its tests, the snappy parity / window / fuzz suites, then decode timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_snsplit; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_snappy_split.py tests/test_gpu_windows.py tests/test_gpu_fuzz.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_split.log 2>&1 || { tail -n 40 $O/pytest_split.log; exit 1; }
tail -n 3 $O/pytest_split.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k snappy -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_parity.log 2>&1 || { tail -n 40 $O/pytest_parity.log; exit 1; }
tail -n 2 $O/pytest_parity.log
for k in 256 512 1024 128; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k$k -o run -- python3 tools/prof_kernels.py --codec snappy --corpus mixed --chunk-kib $k --mib 1024 --reps 5 --decompress > $O/k$k.log 2>&1 || exit 1
done
python3 - $O <<'PY'
import sqlite3, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/k*/*.db')):
    c = sqlite3.connect(f)
    rows = c.execute("select name, count(*), avg(end-start)/1e6 from kernels where name like 'lzh_%' group by name").fetchall()
    print(f.split('/')[-2], [(r[0], r[1], round(r[2], 3)) for r in rows], 'sum', round(sum(r[2] for r in rows if 'decompress' in r[0] or 'snappy' in r[0]), 3))
PY
