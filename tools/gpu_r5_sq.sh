#!/bin/bash
# Round 5 SQ counters on the current build: the 3D tracer (config 4, cube
# 11^2 + L3 and 20^2 + L4), C5 band 0 at 1e9 rays, and method=:direct D2.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_sq3d.sh sq3d_r5_L3 --ndim 11 --level 3 > gpurun_out/sq3d_r5_L3.txt 2>&1 || { tail gpurun_out/sq3d_r5_L3.txt; exit 1; }
bash tools/gpu_sq3d.sh sq3d_r5_L4 --ndim 20 --level 4 > gpurun_out/sq3d_r5_L4.txt 2>&1 || { tail gpurun_out/sq3d_r5_L4.txt; exit 1; }
grep "per wave-ray\|lane\|wait" gpurun_out/sq3d_r5_L3.txt | grep -v "^  SQ_[A-Z_0-9]*  " ; grep "VMEM_RD\|INSTS_VALU \|lane" gpurun_out/sq3d_r5_L3.txt gpurun_out/sq3d_r5_L4.txt
bash tools/gpu_sq_any.sh c5b0_r5 trace_exchange_kernel 999956940 python3 $PWD/tools/bench_configs.py --only C5 \
  --rays 1e9 --steps 1 --bins 0 --no-ramp > gpurun_out/sq_c5b0_r5.log 2>&1 || { tail gpurun_out/sq_c5b0_r5.log; exit 1; }
grep "lane\|SQ_INSTS_VALU \|SQ_INSTS_SALU" gpurun_out/sq_c5b0_r5.log
bash tools/gpu_sq_direct.sh D2 > gpurun_out/sq_direct_D2_r5.log 2>&1 || { tail gpurun_out/sq_direct_D2_r5.log; exit 1; }
grep "lane\|SQ_INSTS_VALU " gpurun_out/sq_direct_D2_r5.log
timeout -k 10 300 python tools/bench_direct.py > gpurun_out/direct_r5.log 2>&1 || { tail gpurun_out/direct_r5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/direct_r5.log
