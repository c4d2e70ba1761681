#!/bin/bash
# tools/full_gpu.sh TAG -- GPU round check: parity suite, smoke, bench line, rocprof kernel stats.
# Everything lands in gpurun_out/TAG/. Steps chained with && (stop at the first failure).
tag=${1:-run}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 \
&& timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 \
&& timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err \
&& (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$out/bench_prof.json 2> $GRAFT_REPO_ROOT/$out/bench_prof.err)
rc=$?
echo "rc=$rc"
tail -3 $out/pytest_gpu.log
cat $out/bench.json
exit $rc
