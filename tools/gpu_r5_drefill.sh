#!/bin/bash
# Round 5: direct-method refill batch (16 in-tree, 12, 24) on D1-D3.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
A=raytraceheattransfer.jl_amd/csrc/_ab
for r in 1 2; do
  for v in "r16 raytraceheattransfer.jl_amd/csrc/_build/librthx.so" "r12 $A/dr12/librthx.so" "r24 $A/dr24/librthx.so"; do
    set -- $v
    RTHX_LIB=$2 timeout -k 10 300 python tools/bench_direct.py --cpu-rays 0 > gpurun_out/drefill_$1.log 2>&1 || { tail gpurun_out/drefill_$1.log; exit 1; }
    grep "^D" gpurun_out/drefill_$1.log | cut -c1-100 | sed "s/^/$1 /" | tee -a gpurun_out/ab_drefill.log
  done
done
