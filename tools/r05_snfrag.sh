# snappy decode, mixed 1 GiB, at -b64 / -b256 / -b1024 (the fragment-parallel ceiling for -b256 decode)
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_snfrag; mkdir -p $O
export TMPDIR=/tmp
for k in 64 256 1024; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k$k -o run -- python3 tools/prof_kernels.py --codec snappy --corpus mixed --chunk-kib $k --mib 1024 --reps 5 --decompress > $O/k$k.log 2>&1 || exit 1
done
python3 - $O <<'PY'
import sqlite3, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/k*/*.db')):
    c = sqlite3.connect(f)
    rows = c.execute("select name, count(*), avg(end-start)/1e6 from kernels where name like 'lzh_decompress%' group by name").fetchall()
    print(f.split('/')[-2], [(r[0], r[1], round(r[2], 3)) for r in rows])
PY
