#!/bin/bash
# tools/exp_build.sh NAME "-DFLAG ..." -- build liblzbench_hip.so with extra defines into build/exp/NAME/
# (kernel experiments; run with LZH_LIB=build/exp/NAME/liblzbench_hip.so)
# ONLY="lz4c_hip ..." compiles just those files with the flags and links the in-tree objects (build/obj, from
# lzbench_amd/csrc/Makefile) for the rest
set -e
name=$1; flags=$2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/build/exp/$name
mkdir -p $out
cd $root/lzbench_amd/csrc
objs=""
for f in lz4c_hip snappyc_hip decode_hip pack_hip zstdc_hip frame_hip; do
  # per-file flags as in the Makefile; SCHED_<file> (e.g. SCHED_decode_hip) overrides one file's
  case $f in
    lz4c_hip) sf="-mllvm -amdgpu-sched-strategy=max-memory-clause" ;;
    snappyc_hip) sf="-mllvm -amdgpu-sched-strategy=max-memory-clause" ;;
    zstdc_hip) sf="-mllvm -amdgpu-atomic-optimizer-strategy=None" ;;
    decode_hip) sf="-mllvm -amdgpu-sched-strategy=max-ilp" ;;
    *) sf="" ;;
  esac
  v=SCHED_$f; [ -n "${!v+x}" ] && sf="${!v}"
  if [ -n "$ONLY" ] && [[ " $ONLY " != *" $f "* ]]; then objs="$objs $root/build/obj/$f.o"; continue; fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $sf $flags -c $f.hip -o $out/$f.o &
  objs="$objs $out/$f.o"
done
if [ -n "$ONLY" ]; then cp $root/build/obj/api.o $root/build/obj/datagen.o $out/; else
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $flags -x hip -c api.cpp -o $out/api.o &
gcc -O2 -fPIC -c datagen.c -o $out/datagen.o &
fi
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/liblzbench_hip.so $objs $out/api.o $out/datagen.o -lm -pthread -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo built $out/liblzbench_hip.so
