#!/bin/bash
# 3D tracer A/B over librthx variants (config 4, 1e8 rays).
set -o pipefail
for v in "$@"; do
  if [ "$v" = main ]; then lib=$PWD/raytraceheattransfer.jl_amd/csrc/_build/librthx.so; else lib=$PWD/raytraceheattransfer.jl_amd/csrc/_variants/$v/librthx.so; fi
  echo "== $v"
  RTHX_LIB=$lib timeout -k 10 120 python tools/bench_trace3d.py --ndim 10 --level 3 --cpu-rows 0 --steps 4 2>&1 | grep config4 | sed 's/BVH.*kernel/kernel/' || exit 1
done
