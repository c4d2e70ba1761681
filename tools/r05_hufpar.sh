# zstd decode: long Huffman streams a wave each (lzh_zstd_hufpar_kernel): zstd GPU tests, then decode timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05_hufpar}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for m in 512 1024; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/zdec_$m -o run -- python3 tools/prof_kernels.py --codec zstd --level 1 --corpus mixed --chunk-kib 128 --mib $m --reps 3 --decompress > $O/zdec_$m.log 2>&1 || exit 1
done
python3 - $O <<'PY'
import sqlite3, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/zdec_*/*.db')):
    c = sqlite3.connect(f)
    rows = c.execute("select name, count(*), avg(end-start)/1e6 from kernels where name like 'lzh_zstd%' and name not like '%match%' and name not like '%entropy%' group by name order by 3 desc").fetchall()
    print(f.split('/')[-2], [(r[0][9:], r[1], round(r[2], 3)) for r in rows], 'decode sum', round(sum(r[2] for r in rows), 3))
PY
