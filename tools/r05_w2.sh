cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_w2; mkdir -p $O
echo base; timeout -k 5 60 python -u tools/rows_diff.py lz4 64 128 text 1 1 > $O/base.log 2>&1; echo rc=$?; cat $O/base.log | grep -v amdgpu
echo walk2; LZH_LIB=$GRAFT_REPO_ROOT/build/exp/walk2/liblzbench_hip.so timeout -k 5 60 python -u tools/rows_diff.py lz4 64 128 text 1 1 > $O/w2.log 2>&1; echo rc=$?; cat $O/w2.log | grep -v amdgpu
