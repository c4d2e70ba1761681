# round 6 call 5: where the register-window parse kernels lose time: P-side sources per batch (stats / clock builds),
# LZ4 register window at 9 vs 10 waves per CU (lzocc9), snappy ring at 3 vs 4 waves per CU (snocc3)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_e; mkdir -p $O
timeout -k 10 120 python tools/lz4_stats.py text json > $O/lz4_stats.txt 2>&1 || { tail $O/lz4_stats.txt; exit 1; }
grep -v amdgpu.ids $O/lz4_stats.txt
for v in snclk snclk0; do for c in json mixed; do
  LZH_LIB=build/exp/$v/liblzbench_hip.so timeout -k 10 120 python tools/sn_clk.py $c 64 512 > $O/${v}_$c.txt 2>&1 || { tail $O/${v}_$c.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $O/${v}_$c.txt
done; done
AB_CORPORA=text timeout -k 10 200 bash tools/ab.sh lzocc9 base > $O/ab_lzocc.log 2>&1 || { tail $O/ab_lzocc.log; exit 1; }
cat $O/ab_lzocc.log
PROF_ARGS="--codec snappy" AB_CORPORA="json" timeout -k 10 300 bash tools/ab.sh snrw0 snocc3 > $O/ab_snocc.log 2>&1 || { tail $O/ab_snocc.log; exit 1; }
cat $O/ab_snocc.log
