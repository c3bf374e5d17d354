#!/bin/bash
# Round 5 diagnostic: the 3D box-hull kernel with its walks removed (wrong
# counts; timing and SQ counters only) against the in-tree build.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
NW=raytraceheattransfer.jl_amd/csrc/_ab/nowalk/librthx.so
for v in "full raytraceheattransfer.jl_amd/csrc/_build/librthx.so" "nowalk $NW"; do
  set -- $v
  RTHX_LIB=$2 timeout -k 10 200 python tools/bench_trace3d.py --ndim 11 --level 3 --cpu-rows 0 > gpurun_out/t3diag_$1.log 2>&1 || { tail gpurun_out/t3diag_$1.log; exit 1; }
  echo "$1: $(grep -o 'kernel [0-9.]* ms ([0-9.]* Grays/s)' gpurun_out/t3diag_$1.log)"
done
RTHX_LIB=$NW bash tools/gpu_sq3d.sh sq3d_nowalk --ndim 11 --level 3 > gpurun_out/sq3d_nowalk.txt 2>&1 || { tail gpurun_out/sq3d_nowalk.txt; exit 1; }
grep "SQ_INSTS_VALU \|VMEM_RD\|lane\|wait" gpurun_out/sq3d_nowalk.txt
