#!/bin/bash
# Round 5: 3D tracer refill batch (16 in-tree, 32, 48) and the refill loop
# (a ray that ends at its hull hit is tallied and the lane takes the next at
# once) -- 3D parity on the loop build, then config-4 A/B.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
A=raytraceheattransfer.jl_amd/csrc/_ab
RTHX_LIB=$A/loop32/librthx.so timeout -k 10 600 python -u -m pytest tests/test_gpu_trace3d.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pt_t3loop.log 2>&1 || { tail -30 gpurun_out/pt_t3loop.log; exit 1; }
tail -1 gpurun_out/pt_t3loop.log
bash tools/gpu_t3_lib_ab.sh refill raytraceheattransfer.jl_amd/csrc/_build/librthx.so $A/r32/librthx.so $A/r48/librthx.so \
  $A/loop16/librthx.so $A/loop32/librthx.so > /dev/null || exit 1
grep -o "^[a-z0-9_]* config4 cube [0-9x]*/face + icosphere L[0-9]\|kernel [0-9.]* ms ([0-9.]* Grays/s)" gpurun_out/t3ab_refill.log | paste - -
