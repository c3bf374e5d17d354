#!/bin/bash
# Round 5: parked ends in the MLAT kernels -- the MLAT / C5 parity tests on
# the in-tree build, then an A/B of the pass and park thresholds on C5 bands
# 0 and 4 at 1e9 rays (base = the build before parking).
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
A=raytraceheattransfer.jl_amd/csrc/_ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "multi_polygon or coarse_lds or c5 or split_part or spectral or mlat or layer" --timeout 400 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pt_park.log 2>&1 || { tail -40 gpurun_out/pt_park.log; exit 1; }
tail -1 gpurun_out/pt_park.log
bash tools/gpu_ab_c5.sh park "0 4" $A/base/librthx.so raytraceheattransfer.jl_amd/csrc/_build/librthx.so \
  $A/r16/librthx.so $A/r24/librthx.so $A/r24p32/librthx.so $A/r16p48/librthx.so
