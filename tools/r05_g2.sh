set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_b; mkdir -p $O
timeout -k 10 200 python tools/lz4_diff.py text 64 1 1024 12345 > $O/diff_text1g.log 2>&1; rc=$?; tail -4 $O/diff_text1g.log
case $rc in 124|137|134|139) exit $rc;; esac
STATS_MIB=512 timeout -k 10 120 python tools/lz4_stats.py --parse2 text json > $O/stats2.log 2>&1; rc=$?; cat $O/stats2.log | grep -v amdgpu.ids
case $rc in 124|137|134|139) exit $rc;; esac
STATS_MIB=512 LZH_LIB=build/exp/p1/liblzbench_hip.so timeout -k 10 120 python tools/lz4_stats.py text > $O/stats1.log 2>&1; cat $O/stats1.log | grep -v amdgpu.ids
PROF_ARGS="--corpus text" bash tools/pmc_inst.sh gpurun_out/r05_b/pmc base p1 > $O/pmc.txt 2>&1; cat $O/pmc.txt | grep -E "==|parse|WAVE|INSTS|WAIT|ACTIVE|BANK"
