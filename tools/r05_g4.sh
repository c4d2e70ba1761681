set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05_d; mkdir -p $O
for r in 1 2; do for v in base p1 pr1 pr3; do
  if [ $v = base ]; then LL=""; else LL=build/exp/$v/liblzbench_hip.so; fi
  echo -n "r$r $v text: "; LZH_LIB=$LL timeout -k 10 120 python tools/prof_kernels.py --mib 1024 --reps 5 --corpus text 2>&1 | grep -v amdgpu.ids | tail -1 || exit 5
done; done > $O/ab.txt 2>&1; cat $O/ab.txt
PROF_ARGS="--corpus text" bash tools/pmc_inst.sh gpurun_out/r05_d/pmc base > $O/pmc.txt 2>&1; grep -A16 "parse2_kernel" $O/pmc.txt
