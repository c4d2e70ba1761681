# zstd decode stats build (LZH_ZSTD_STATS): per-wave steps / clocks of the seq and huf kernels at 512 MiB / 1 GiB
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_zst; mkdir -p $O
for m in 512 1024; do
  LZH_LIB=build/exp/zst/liblzbench_hip.so timeout -k 10 120 python3 tools/prof_kernels.py --codec zstd --level 1 --corpus mixed --chunk-kib 128 --mib $m --reps 10 --decompress > $O/zst_$m.log 2>&1 || exit 1
  grep -a "seq kernel" $O/zst_$m.log | sed "s/.*steps/steps/" || true
done
