# LZ4 parse with the 8-byte seed window (build/exp/seed8, -DLZH_LZ4_SEED8=1): parity at 1 GiB, time A/B
# against the in-tree parse, instruction / stall counters and HBM traffic
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_seed8; mkdir -p $O
export TMPDIR=/tmp
S8=$GRAFT_REPO_ROOT/build/exp/seed8/liblzbench_hip.so
LZH_LIB=$S8 timeout -k 10 300 python -u tools/lz4_diff.py text 64 1 1024 > $O/diff_text.log 2>&1 && \
LZH_LIB=$S8 timeout -k 10 300 python -u tools/lz4_diff.py json 64 1 1024 > $O/diff_json.log 2>&1 || { tail $O/diff_*.log; exit 1; }
for v in base seed8; do
  ( if [ $v != base ]; then export LZH_LIB=$S8; fi
    for c in text json; do
      timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/t_${v}_$c -o run -- python3 tools/prof_kernels.py --codec lz4 --corpus $c --mib 1024 --reps 5 > $O/t_${v}_$c.log 2>&1 || exit 1
    done ) || exit 1
done
bash tools/pmc_inst.sh $O/inst base seed8 > $O/inst.txt 2>&1 && \
LZH_LIB=$S8 bash tools/pmc_traffic.sh $O/traffic_seed8 lz4 text 64 1 1024 > /dev/null || exit 1
for m in 512 1024; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/zdec_$m -o run -- python3 tools/prof_kernels.py --codec zstd --level 1 --corpus mixed --chunk-kib 128 --mib $m --reps 3 --decompress > $O/zdec_$m.log 2>&1 || exit 1
done
echo done
