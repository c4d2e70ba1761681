#!/bin/bash
# tools/gpu_round.sh STEP... -- GPU-box steps, each under its own time limit, stopping at the first
# failure; logs and results under gpurun_out/<tag>/ (tag = $LZH_TAG or "run").
#   tests:<pytest args>   python -m pytest -m gpu with the given args (a test file / -k expression)
#   bench                 python bench.py (defaults: N=1, e2e and CPU baseline included)
#   benchq                python bench.py --no-e2e --no-cpu-baseline
#   prof                  rocprofv3 --kernel-trace --stats of benchq
#   ddp2                  one-GPU torchrun world-2 rehearsal of bench.py --gpus 2
#   sweep                 tools/config_sweep.sh into gpurun_out/<tag>/configs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${LZH_TAG:-run}
O=gpurun_out/$T
mkdir -p "$O"
for step in "$@"; do
  echo "== $step $(date +%T)"
  case "$step" in
    tests:*)
      a=${step#tests:}
      timeout -k 10 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $a > "$O/pytest.log" 2>&1
      rc=$?; tail -3 "$O/pytest.log"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$O/bench.json" 2> "$O/bench.err" || { tail "$O/bench.err"; exit 1; }
      cat "$O/bench.json" ;;
    benchq)
      timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline $LZH_BENCH_ARGS > "$O/benchq.json" 2> "$O/benchq.err" || { tail "$O/benchq.err"; exit 1; }
      cat "$O/benchq.json" ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 bench.py --no-e2e --no-cpu-baseline $LZH_BENCH_ARGS > "$O/bench_under_rocprof.json" 2> "$O/prof.err" || { tail "$O/prof.err"; exit 1; }
      find "$O/prof" -name "*kernel_stats.csv" -exec cp {} "$O/run_kernel_stats.csv" \; ;;
    ddp2)
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
        bench.py --gpus 2 --steps 3 --warmup 1 > "$O/ddp2.json" 2> "$O/ddp2.err" || { tail "$O/ddp2.err"; exit 1; }
      cat "$O/ddp2.json" ;;
    sweep)
      timeout -k 10 1100 bash tools/config_sweep.sh "$O/configs" > "$O/sweep.log" 2>&1 || { tail "$O/sweep.log"; exit 1; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
