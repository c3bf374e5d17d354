#!/bin/bash
# Kernel iteration on the GPU box (repo root): the GPU test suite on the
# in-tree build, then an interleaved A/B of librthx.so variants on C2 and on
# C5 band 0 / band 7 at 1e9 rays (tools/ab.py, one process per config).
#   bash tools/gpu_iter.sh TAG lib1.so lib2.so ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > $OUT/pt_$TAG.log 2>&1 || { tail -40 $OUT/pt_$TAG.log; exit 1; }
tail -n 1 $OUT/pt_$TAG.log
timeout -k 10 200 python tools/ab.py --rounds 10 --steps 5 "$@" 2>&1 | grep -v amdgpu.ids | sed "s/^/C2  /" \
  | tee $OUT/ab_$TAG.log || exit 1
for b in 0 7; do
  timeout -k 10 300 python tools/ab.py --c5-bin $b --rays 1000000000 --rounds 3 --steps 2 "$@" 2>&1 \
    | grep -v amdgpu.ids | sed "s/^/C5 band $b  /" | tee -a $OUT/ab_$TAG.log || exit 1
done
