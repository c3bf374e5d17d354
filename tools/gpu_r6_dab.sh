#!/bin/bash
# Direct-method A/B of librthx.so variants (csrc/_ab/<name>) on D1-D3, alternating twice.
#   bash tools/gpu_r6_dab.sh name1 name2 ...
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out
C=raytraceheattransfer.jl_amd/csrc
for r in 1 2; do
for n in "$@"; do
  L=$C/_ab/$n/librthx.so; [ "$n" = "_build" ] && L=$C/_build/librthx.so
  RTHX_LIB=$L timeout -k 10 200 python tools/bench_direct.py --cpu-rays 0 --only D1,D2,D3 2>&1 | grep -v amdgpu.ids | sed "s|^|$n |" | cut -c1-140 || exit 1
done
done
