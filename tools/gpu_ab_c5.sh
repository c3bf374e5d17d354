#!/bin/bash
# A/B of librthx.so variants on C5 bands (one process, interleaved rounds):
#   bash tools/gpu_ab_c5.sh TAG "BINS" lib1.so lib2.so ...
set -o pipefail
TAG=$1; BINS=$2; shift 2
mkdir -p gpurun_out
for b in $BINS; do
  timeout -k 10 300 python tools/ab.py --c5-bin $b --rays 1000000000 --rounds 3 --steps 2 "$@" 2>&1 \
    | grep -v amdgpu.ids | sed "s/^/band $b  /" | tee -a gpurun_out/ab_$TAG.log || exit 1
done
