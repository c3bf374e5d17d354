#!/bin/bash
# A/B of librthx.so variants on the direct-method cases (RTHX_LIB per run),
# then the SQ counters of the in-tree build on one case.
#   bash tools/gpu_direct_ab.sh TAG CASES SQ_CASE lib1.so lib2.so ...
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
TAG=$1; CASES=$2; SQC=$3; shift 3
mkdir -p gpurun_out
for lib in "$@"; do
  RTHX_LIB=$lib timeout -k 10 200 python tools/bench_direct.py --only $CASES --cpu-rays 0 2>&1 | grep -v amdgpu.ids \
    | sed "s|^|$(basename $(dirname $lib)) |" | tee -a gpurun_out/direct_$TAG.log || exit 1
done
if [ -n "$SQC" ]; then bash tools/gpu_sq_direct.sh $SQC > gpurun_out/sq_direct_$TAG.log 2>&1 || exit 1; cat gpurun_out/sq_direct_$TAG.log; fi
