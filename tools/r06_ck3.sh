# round 6 checkpoint 3: per-class instruction counters of the shipping parse kernels (LZ4 text, snappy JSON), three
# rocprofv3 --pmc passes each (tools/pmc_parse.sh), for the per-batch instruction model
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${CK_TAG:-r06_ck}
mkdir -p gpurun_out/$T
bash tools/pmc_parse.sh gpurun_out/$T/pmc_lz4 base > gpurun_out/$T/pmc_lz4.log 2>&1 || { tail gpurun_out/$T/pmc_lz4.log; exit 1; }
PROF_ARGS="--codec snappy --corpus json" bash tools/pmc_parse.sh gpurun_out/$T/pmc_sn base > gpurun_out/$T/pmc_sn.log 2>&1 || { tail gpurun_out/$T/pmc_sn.log; exit 1; }
python3 tools/pmc_summary.py gpurun_out/$T/pmc_lz4/base > gpurun_out/$T/pmc_lz4_summary.txt
python3 tools/pmc_summary.py gpurun_out/$T/pmc_sn/base > gpurun_out/$T/pmc_sn_summary.txt
grep -A24 "lz4_parse_kernel" gpurun_out/$T/pmc_lz4_summary.txt
# the bench line again, now that profiles/traffic_r06_*.json hold the shipping kernels' traffic
timeout -k 10 300 python -u bench.py --no-e2e --no-cpu-baseline > gpurun_out/$T/benchq_traffic.json 2> gpurun_out/$T/benchq_traffic.err || { tail gpurun_out/$T/benchq_traffic.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/$T/benchq_traffic.json'));print(d['value'], d['bit_exact'], d['roofline'])"
