#!/bin/bash
# tools/round_profile.sh TAG -- everything a round's profiles/TAG needs, in one GPU call:
# GPU parity suite, smoke, bench line, rocprofv3 kernel stats of the bench, traffic PMC passes.
tag=${1:-run}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1 || { tail -20 $out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { tail $out/smoke.log; exit 1; }
bash tools/pmc_traffic.sh $out/traffic > $out/traffic.log 2>&1 || { tail $out/traffic.log; exit 1; }
mkdir -p profiles && cp $out/traffic/traffic.json profiles/traffic.json
timeout -k 10 400 python bench.py > $out/bench.json 2> $out/bench.err || { tail $out/bench.err; exit 1; }
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 5 --warmup 2 > $GRAFT_REPO_ROOT/$out/bench_prof.json 2> $GRAFT_REPO_ROOT/$out/bench_prof.err) || exit 1
tail -1 $out/pytest_gpu.log; cat $out/bench.json
