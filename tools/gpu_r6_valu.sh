#!/bin/bash
# Headline VALU trims (round 6): HEAD against the working tree; the GPU
# suite on the new build first (every kernel that shares the device code).
export RTHX_DEV_KNOBS=1
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_valu.log 2>&1 || { tail -30 $OUT/pytest_valu.log; exit 1; }
tail -1 $OUT/pytest_valu.log
C=raytraceheattransfer.jl_amd/csrc
timeout -k 10 400 python tools/ab.py --rounds 20 $C/_ab/head/librthx.so $C/_build/librthx.so 2>&1 | grep -v amdgpu.ids
for L in $C/_ab/head/librthx.so $C/_build/librthx.so; do
  RTHX_LIB=$L timeout -k 10 200 python tools/bench_direct.py --cpu-rays 0 --only D1,D2 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $(dirname $L)) |" | cut -c1-140
done
