# zstd match-kernel phase clocks (LZH_ZSTDC_STATS build): mixed / text at -b128, 256 MiB
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_zcs; mkdir -p $O
for c in mixed text; do
  LZH_LIB=build/exp/zcs/liblzbench_hip.so timeout -k 10 120 python3 tools/zstdc_stats.py $c 128 256 > $O/zcs_$c.log 2>&1 || { cat $O/zcs_$c.log; exit 1; }
  cat $O/zcs_$c.log
done
