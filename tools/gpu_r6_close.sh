#!/bin/bash
# Round 6 closing evidence on HEAD: the full refresh (tools/gpu_r6_final.sh),
# then the direct method's D2 SQ counters.
set -o pipefail
bash tools/gpu_r6_final.sh ${1:-r6c} || exit 1
bash tools/gpu_sq_direct.sh D2 > gpurun_out/sq_direct_D2_${1:-r6c}.log 2>&1 || { tail gpurun_out/sq_direct_D2_${1:-r6c}.log; exit 1; }
cat gpurun_out/sq_direct_D2_${1:-r6c}.log
