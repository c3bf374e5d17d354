#!/bin/bash
# Round 6 direct-method A/B: the direct GPU tests on the working tree, then
# HEAD (_ab/head) against it on D1-D3, alternating twice.
export RTHX_DEV_KNOBS=1
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_direct.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_dir.log 2>&1 || { tail -30 $OUT/pytest_dir.log; exit 1; }
tail -1 $OUT/pytest_dir.log
C=raytraceheattransfer.jl_amd/csrc
for r in 1 2; do
for L in $C/_ab/head/librthx.so $C/_build/librthx.so; do
  RTHX_LIB=$L timeout -k 10 200 python tools/bench_direct.py --cpu-rays 0 --only D1,D2,D3 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $(dirname $L)) |" | cut -c1-140 || exit 1
done
done
