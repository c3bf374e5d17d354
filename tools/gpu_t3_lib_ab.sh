#!/bin/bash
# 3D tracer A/B of librthx.so builds (one process per library and case, two rounds):
#   bash tools/gpu_t3_lib_ab.sh TAG lib1.so lib2.so ...
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for r in 1 2; do
  for L in "$@"; do
    for c in "11 3" "20 4"; do
      nd=${c% *}; lv=${c#* }
      RTHX_LIB=$L timeout -k 10 200 python tools/bench_trace3d.py --ndim $nd --level $lv --cpu-rows 0 2>&1 | grep config4 \
        | sed "s|^|$(basename $(dirname $L)) |" | tee -a gpurun_out/t3ab_$TAG.log || exit 1
    done
  done
done
