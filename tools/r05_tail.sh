# wave-quantisation tail of the LZ4 parse: 7 x 2304 chunks (1008 MiB), 1 GiB, 8 x 2304 (1152 MiB), text -b64
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_tail; mkdir -p $O
export TMPDIR=/tmp
for m in 1008 1024 1152 1008 1024 1152; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/m$m -o run_$RANDOM -- python3 tools/prof_kernels.py --codec lz4 --corpus text --mib $m --reps 5 > $O/m$m.log 2>&1 || exit 1
done
python3 - $O <<'PY'
import sqlite3, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/m*/*.db')):
    c = sqlite3.connect(f)
    rows = c.execute("select name, count(*), avg(end-start)/1e6, min(end-start)/1e6 from kernels where name like 'lzh_lz4_parse%' group by name").fetchall()
    print(f.split('/')[-2], [(r[1], round(r[2], 3), round(r[3], 3)) for r in rows])
PY
