#!/bin/bash
# tools/e2e_cli.sh TAG -- end-to-end (host buffers, PCIe included) lzbench-style runs of the CLI driver on
# 1 GiB synthetic text: hipMemcpy, hip_lz4 -b64, hip_snappy -b256 (mixed), CPU lz4 on a 64 MiB sample
tag=${1:-e2e}; out=gpurun_out/$tag; mkdir -p $out
python - <<'PY'
import lzbench_amd as L
L.datagen("text", 1 << 30, seed=12345).tofile("/tmp/text1g.bin")
L.datagen("mixed", 1 << 30, seed=12345).tofile("/tmp/mixed1g.bin")
L.datagen("text", 64 << 20, seed=12345).tofile("/tmp/text64m.bin")
PY
timeout -k 10 300 ./lzbench_amd/lzbench_hip -ehipMemcpy/hip_lz4 -b64 -i3,3 -t0,0 /tmp/text1g.bin > $out/text_lz4.txt 2>&1 || exit 1
timeout -k 10 300 ./lzbench_amd/lzbench_hip -ehip_snappy -b256 -i3,3 -t0,0 /tmp/mixed1g.bin > $out/mixed_snappy.txt 2>&1 || exit 1
timeout -k 10 300 ./lzbench_amd/lzbench_hip -elz4 -b64 -i1,1 -t0,0 /tmp/text64m.bin > $out/cpu_lz4.txt 2>&1 || exit 1
cat $out/*.txt
