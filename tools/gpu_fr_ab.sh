#!/bin/bash
# frames tests + bench on the in-tree library, then decoder A/B of experiment builds
bash tools/gpu_frames.sh $1 || exit 1
shift
bash tools/dec_ab.sh base "$@"
