#!/bin/bash
# Round 5: the 3D tracer's draws from 7-round Philox blocks (in-tree) --
# 3D GPU tests and known answers, then config 4 against the 10-round build
# (csrc/_ab/base).
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_trace3d.py tests/test_gpu_known_answers.py -m gpu -x -q --timeout 400 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pt_t3p7.log 2>&1 || { tail -30 gpurun_out/pt_t3p7.log; exit 1; }
tail -1 gpurun_out/pt_t3p7.log
bash tools/gpu_t3_lib_ab.sh t3p7 raytraceheattransfer.jl_amd/csrc/_ab/base/librthx.so raytraceheattransfer.jl_amd/csrc/_build/librthx.so > /dev/null || exit 1
grep -o "^[a-z0-9_]* config4 cube [0-9x]*/face + icosphere L[0-9]\|kernel [0-9.]* ms ([0-9.]* Grays/s)" gpurun_out/t3ab_t3p7.log | paste - -
