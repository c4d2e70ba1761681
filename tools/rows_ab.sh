# tools/rows_ab.sh VARIANT CODEC "CORPUS:CHUNK_KIB ..." -- parity (rows vs the reference at 1 GiB) and a
# compress-kernel A/B (in-tree vs build/exp/VARIANT, alternating, two rounds), rocprofv3 kernel traces
set -o pipefail
cd $GRAFT_REPO_ROOT
V=$1; C=$2; W=$3
O=gpurun_out/ab_$V; mkdir -p $O
export TMPDIR=/tmp
LIB=$GRAFT_REPO_ROOT/build/exp/$V/liblzbench_hip.so
for w in $W; do c=${w%%:*}; k=${w##*:}
  LZH_LIB=$LIB timeout -k 10 300 python -u tools/rows_diff.py $C $k 256 $c 1 1 > $O/diff_$c.log 2>&1 || { tail $O/diff_$c.log; exit 1; }
  grep -q "bad chunks 0" $O/diff_$c.log || { echo "parity FAILED $c"; cat $O/diff_$c.log; exit 1; }
done
for r in 1 2; do for v in base $V; do for w in $W; do c=${w%%:*}; k=${w##*:}
  ( if [ $v != base ]; then export LZH_LIB=$LIB; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/t${r}_${v}_$c -o run -- python3 tools/prof_kernels.py --codec $C --corpus $c --chunk-kib $k --mib 1024 --reps 5 > $O/t${r}_${v}_$c.log 2>&1 ) || exit 1
done; done; done
python3 - $O <<'PY'
import sqlite3, glob, sys
for f in sorted(glob.glob(sys.argv[1] + '/t*/run_results.db')):
    c = sqlite3.connect(f)
    rows = c.execute("select name, count(*), avg(end-start)/1e6 from kernels where name like 'lzh%' group by name order by 3 desc limit 2").fetchall()
    print(f.split('/')[-2], [(r[0], round(r[2], 3)) for r in rows])
PY
