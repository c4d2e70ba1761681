# decoder dword emission (groups::emit_group4): the GPU suite on the default build, then decode A/B
# against the two-byte emitter (build/exp/d0) and the 8-wave-capped build (build/exp/d8)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_dec4; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -n 30 $O/pytest.log; exit 1; }
tail -n 2 $O/pytest.log
for v in def d0 d8; do
  if [ $v != def ]; then export LZH_LIB=$GRAFT_REPO_ROOT/build/exp/$v/liblzbench_hip.so; fi
  for w in "lz4 text 64" "lz4 json 64" "snappy mixed 256" "snappy json 64"; do set -- $w
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_${v}_$1_$2 -o run -- python3 tools/prof_kernels.py --codec $1 --corpus $2 --chunk-kib $3 --mib 1024 --reps 5 --decompress > $O/ab_${v}_$1_$2.log 2>&1 || exit 1
  done
done
echo done
