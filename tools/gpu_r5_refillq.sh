#!/bin/bash
# Round 5: MLAT pass threshold (RTHX_REFILL_Q 40 in-tree, 32, 48) re-measured
# on C5 bands 0 / 4 at 1e9 and 1e8 rays.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
A=raytraceheattransfer.jl_amd/csrc/_ab
bash tools/gpu_ab_c5.sh refillq "0 4" raytraceheattransfer.jl_amd/csrc/_build/librthx.so $A/q32/librthx.so $A/q48/librthx.so || exit 1
for b in 0 4; do
  timeout -k 10 300 python tools/ab.py --c5-bin $b --rays 100000000 --rounds 5 --steps 3 raytraceheattransfer.jl_amd/csrc/_build/librthx.so \
    $A/q32/librthx.so $A/q48/librthx.so 2>&1 | grep -v amdgpu.ids | sed "s/^/1e8 band $b  /" | tee -a gpurun_out/ab_refillq.log || exit 1
done
