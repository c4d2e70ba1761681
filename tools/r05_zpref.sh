# zstd match kernel: first-batch loads issued with the table fills (LZH_ZSTD_PREF) -- compress parity tests,
# then A/B against the -DLZH_ZSTD_PREF=0 build and rocprof kernel times
set -o pipefail
cd $GRAFT_REPO_ROOT
O=${O:-gpurun_out/r05_zpref}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd_compress.py tests/test_zstd_golden.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -n 40 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
timeout -k 10 600 bash tools/zstdc_ab.sh base ${AB:-nopref} > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 tools/prof_kernels.py --codec zstd --level 1 --corpus mixed --chunk-kib 128 --mib 512 --reps 3 > $O/prof.log 2>&1 || exit 1
python3 - $O <<'PY'
import sqlite3, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/prof/*.db')):
    c = sqlite3.connect(f)
    print([(r[0], r[1], round(r[2], 3)) for r in c.execute("select name, count(*), avg(end-start)/1e6 from kernels where name like 'lzh_zstd_match%' or name like 'lzh_zstd_entropy%' group by name").fetchall()])
PY
