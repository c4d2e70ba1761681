set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_f; mkdir -p $O
LZH_LIB=build/exp/snclk/liblzbench_hip.so timeout -k 10 120 python tools/sn_clk.py json 64 512 > $O/snclk.log 2>&1 || { cat $O/snclk.log; exit 3; }
LZH_LIB=build/exp/snclk/liblzbench_hip.so timeout -k 10 120 python tools/sn_clk.py mixed 256 512 >> $O/snclk.log 2>&1 || { cat $O/snclk.log; exit 3; }
grep -v amdgpu.ids $O/snclk.log
bash tools/gpu_suite.sh r05_suite1
