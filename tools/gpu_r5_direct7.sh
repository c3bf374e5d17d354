#!/bin/bash
# Round 5: a direct-method change (in-tree) -- direct
# parity and known answers, then D1-D3 against the build before (csrc/_ab/base).
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_direct.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pt_direct7.log 2>&1 || { tail -30 gpurun_out/pt_direct7.log; exit 1; }
tail -1 gpurun_out/pt_direct7.log
for r in 1 2; do
  for v in "base raytraceheattransfer.jl_amd/csrc/_ab/base/librthx.so" "new raytraceheattransfer.jl_amd/csrc/_build/librthx.so"; do
    set -- $v
    RTHX_LIB=$2 timeout -k 10 300 python tools/bench_direct.py --cpu-rays 0 > gpurun_out/direct7_$1.log 2>&1 || { tail gpurun_out/direct7_$1.log; exit 1; }
    grep "^D" gpurun_out/direct7_$1.log | cut -c1-110 | sed "s/^/$1 /" | tee -a gpurun_out/ab_direct7.log
  done
done
