#!/bin/bash
# 3D tracer: GPU tests, then config 4 (L3, L4) under each setting of one
# environment knob (e.g. RTHX_T3_GHIST, RTHX_T3_SPLIT_TARGET; "auto" = unset).
#   bash tools/gpu_t3_env.sh TAG VAR "auto 0 1"
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
TAG=$1; VAR=$2; SETS=$3
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_trace3d.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pt_$TAG.log 2>&1 || { tail -40 gpurun_out/pt_$TAG.log; exit 1; }
tail -n 1 gpurun_out/pt_$TAG.log
for v in $SETS; do
  if [ $v = auto ]; then unset $VAR; else export $VAR=$v; fi
  timeout -k 10 200 python tools/bench_trace3d.py --ndim 10 --level 3 --cpu-rows 0 2>&1 | grep config4 | sed "s|^|$VAR=$v |" | tee -a gpurun_out/t3_$TAG.log || exit 1
  timeout -k 10 200 python tools/bench_trace3d.py --ndim 20 --level 4 --cpu-rows 0 2>&1 | grep config4 | sed "s|^|$VAR=$v |" | tee -a gpurun_out/t3_$TAG.log || exit 1
done
