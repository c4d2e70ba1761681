# round 6 call 26: the LZ4 parse kernel under other machine schedulers (the file is built with max-ilp): the default
# (sdef), iterative-ilp (silp), max-memory-clause (smmc) -- A/B against the head
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r06_za; mkdir -p $O
AB_CORPORA="text json" AB_ROUNDS=2 timeout -k 10 700 bash tools/ab.sh head sdef silp smmc > $O/ablz.log 2>&1 || { tail $O/ablz.log; exit 1; }
cat $O/ablz.log
