set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_e; mkdir -p $O
PROF_ARGS="--codec snappy --corpus json" bash tools/pmc_inst.sh gpurun_out/r05_e/snjson base > $O/snjson.txt 2>&1 || exit 3
PROF_ARGS="--codec snappy --corpus mixed --chunk-kib 256" bash tools/pmc_inst.sh gpurun_out/r05_e/snmixed base > $O/snmixed.txt 2>&1 || exit 3
PROF_ARGS="--corpus text --decompress" bash tools/pmc_inst.sh gpurun_out/r05_e/dec base > $O/dec.txt 2>&1 || exit 3
PROF_ARGS="--codec zstd --level 1 --corpus mixed --chunk-kib 128" bash tools/pmc_inst.sh gpurun_out/r05_e/zstd base > $O/zstd.txt 2>&1 || exit 3
for f in snjson snmixed dec zstd; do echo "=== $f"; python3 tools/pmc_summary.py gpurun_out/r05_e/$f/base; done > $O/summary.txt
cat $O/summary.txt | head -150
