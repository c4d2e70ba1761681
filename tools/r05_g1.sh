set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_a; mkdir -p $O
timeout -k 10 90 python -c "
import sys; sys.path.insert(0,'.'); sys.path.insert(0,'tests')
import lzbench_amd as L, oracle_lib as O, numpy as np
for corpus in ('text','json','random','mixed'):
    d = L.datagen(corpus, 3*65536+777, seed=5)
    p, cs = L.compress_chunks(d, 'lz4', 65536, 1)
    op, ocs = O.compress_chunks(d, 'lz4', 65536, 1)
    print(corpus, len(p), len(op), bool((cs==ocs).all()) and bool((p==op).all()), flush=True)
" > $O/small.log 2>&1; rc=$?; cat $O/small.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python tools/lz4_diff.py text 64 > $O/diff_text.log 2>&1 || { tail $O/diff_text.log; exit 3; }
tail -3 $O/diff_text.log
timeout -k 10 120 python tools/lz4_diff.py json 64 > $O/diff_json.log 2>&1 || { tail $O/diff_json.log; exit 3; }
tail -3 $O/diff_json.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stress.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
case $rc in 124|137|134|139) exit $rc;; esac
for r in 1 2; do for v in base p1; do
  if [ $v = base ]; then LL=""; else LL=build/exp/p1/liblzbench_hip.so; fi
  for c in text json; do echo -n "r$r $v $c: "; LZH_LIB=$LL timeout -k 10 120 python tools/prof_kernels.py --mib 1024 --reps 5 --corpus $c 2>&1 | grep -v amdgpu.ids | tail -1 || exit 5; done
done; done > $O/ab.txt 2>&1; cat $O/ab.txt
