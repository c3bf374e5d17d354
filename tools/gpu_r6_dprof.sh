#!/bin/bash
# Per-region lane counts of the direct kernel (diagnostic build _ab/prof, RTHX_DIRECT_PROF=1).
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out
RTHX_LIB=raytraceheattransfer.jl_amd/csrc/_ab/prof/librthx.so timeout -k 10 200 python tools/bench_direct.py --cpu-rays 0 --rays 1e7 --steps 1 --only D2,D1,D3 > gpurun_out/dprof.log 2>&1 || { tail -20 gpurun_out/dprof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/dprof.log
