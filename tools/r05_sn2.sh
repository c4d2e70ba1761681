# snappy two-wave parse: parity (rows vs the reference) then A/B against the one-wave parse (build/exp/sn1)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_sn2; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 python -u tools/rows_diff.py snappy 64 256 json 0 1 > $O/diff_json64.log 2>&1 && \
timeout -k 10 240 python -u tools/rows_diff.py snappy 256 256 mixed 0 1 > $O/diff_mixed256.log 2>&1 && \
timeout -k 10 240 python -u tools/rows_diff.py snappy 64 128 text 0 1 > $O/diff_text64.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k snappy -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 && \
for v in 2 1; do
  if [ $v = 1 ]; then export LZH_LIB=$GRAFT_REPO_ROOT/build/exp/sn1/liblzbench_hip.so; fi
  for w in "json 64" "mixed 256" "text 64"; do set -- $w
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p${v}_$1 -o run -- python3 tools/prof_kernels.py --codec snappy --corpus $1 --chunk-kib $2 --mib 1024 --reps 5 > $O/ab_v${v}_$1.log 2>&1 || exit 1
  done
done
echo done
