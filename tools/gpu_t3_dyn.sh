#!/bin/bash
# 3D tracer A/B: workgroup size (library variants built by tools/variant_make.sh
# with T3_FLAGS=-DRTHX_T3_THREADS=N) x top nodes in dynamic LDS (RTHX_T3_DYNTOP,
# breadth-first top of RTHX_T3_BFS_TOP nodes, at most RTHX_T3_DYNTOP_MAX).
#   bash tools/gpu_t3_dyn.sh TAG "lib1 lib2 ..." "ENV1;ENV2;..."   (lib "-" = the default build)
set -o pipefail
TAG=$1; LIBS=$2
IFS=';' read -ra ENVS <<< "$3"
mkdir -p gpurun_out
for lib in $LIBS; do
  for E in "${ENVS[@]}"; do
    envs=""; [ "$E" != "-" ] && envs="$E"
    L=""; [ "$lib" != "-" ] && L="RTHX_LIB=raytraceheattransfer.jl_amd/csrc/_ab/$lib/librthx.so"
    for nl in "11 3" "20 4"; do
      set -- $nl
      env $L $envs timeout -k 10 200 python tools/bench_trace3d.py --ndim $1 --level $2 --cpu-rows 0 2>&1 | grep config4 \
        | sed "s|^|$lib $E |" | tee -a gpurun_out/t3dyn_$TAG.log || exit 1
    done
  done
done
