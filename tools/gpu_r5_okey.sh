#!/bin/bash
# Round 5: Philox round keys formed per block (RTHX_PHILOX_OPAQUE_KEY=1,
# csrc/_ab/okey) against the hoisted keys (in-tree) on C2, C3 and C5.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
IN=raytraceheattransfer.jl_amd/csrc/_build/librthx.so
OK=raytraceheattransfer.jl_amd/csrc/_ab/okey/librthx.so
timeout -k 10 300 python tools/ab.py --rounds 10 $IN $OK 2>&1 | grep -v amdgpu.ids | sed 's/^/C2  /' | tee gpurun_out/ab_okey.log || exit 1
timeout -k 10 300 python tools/ab.py --rounds 10 --ndim 51 $IN $OK 2>&1 | grep -v amdgpu.ids | sed 's/^/51x51  /' | tee -a gpurun_out/ab_okey.log || exit 1
bash tools/gpu_ab_c5.sh okey "0" $IN $OK || exit 1
