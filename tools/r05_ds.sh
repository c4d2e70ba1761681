cd $GRAFT_REPO_ROOT
for b in decst decst0; do for w in "lz4 text" "lz4 json" "snappy mixed"; do
  LZH_LIB=$GRAFT_REPO_ROOT/build/exp/$b/liblzbench_hip.so STATS_KIB=$([ "$w" = "snappy mixed" ] && echo 256 || echo 64) timeout -k 10 120 python -u tools/dec_stats.py $w || exit 1
done; done
