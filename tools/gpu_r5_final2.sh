#!/bin/bash
# Round 5 closing evidence: the full refresh (gpu_r5_final.sh), the strong
# shards, the direct method (D1-D3) and the 3D / C5 SQ counters.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
TAG=${1:-r5c}
bash tools/gpu_r5_final.sh $TAG || exit 1
timeout -k 10 400 bash tools/gpu_strong.sh > gpurun_out/strong_$TAG.log 2>&1 || { tail gpurun_out/strong_$TAG.log; exit 1; }
cat gpurun_out/strong_$TAG.log
timeout -k 10 300 python tools/bench_direct.py > gpurun_out/direct_$TAG.log 2>&1 || { tail gpurun_out/direct_$TAG.log; exit 1; }
grep "^D" gpurun_out/direct_$TAG.log | cut -c1-120
bash tools/gpu_sq_direct.sh D2 > gpurun_out/sq_direct_D2_$TAG.log 2>&1 || { tail gpurun_out/sq_direct_D2_$TAG.log; exit 1; }
bash tools/gpu_sq3d.sh sq3d_${TAG}_L3 --ndim 11 --level 3 > gpurun_out/sq3d_${TAG}_L3.txt 2>&1 || { tail gpurun_out/sq3d_${TAG}_L3.txt; exit 1; }
bash tools/gpu_sq_any.sh c5b0_$TAG trace_exchange_kernel 999956940 python3 $PWD/tools/bench_configs.py --only C5 \
  --rays 1e9 --steps 1 --bins 0 --no-ramp > gpurun_out/sq_c5b0_$TAG.log 2>&1 || { tail gpurun_out/sq_c5b0_$TAG.log; exit 1; }
grep "lane\|SQ_INSTS_VALU " gpurun_out/sq_direct_D2_$TAG.log gpurun_out/sq3d_${TAG}_L3.txt gpurun_out/sq_c5b0_$TAG.log
