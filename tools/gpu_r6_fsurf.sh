#!/bin/bash
# LAT wall hits from D.f_surf (working tree) against HEAD's boundary arrays:
# the GPU suite on the new build, then headline and direct D1/D2 timings.
export RTHX_DEV_KNOBS=1
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_fsurf.log 2>&1 || { tail -30 $OUT/pytest_fsurf.log; exit 1; }
tail -1 $OUT/pytest_fsurf.log
A=raytraceheattransfer.jl_amd/csrc/_ab/head/librthx.so
B=raytraceheattransfer.jl_amd/csrc/_build/librthx.so
timeout -k 10 300 python tools/ab.py --rounds 20 $A $B 2>&1 | grep -v amdgpu.ids
for L in $A $B; do
  RTHX_LIB=$L timeout -k 10 200 python tools/bench_direct.py --cpu-rays 0 --only D1,D2 2>&1 | grep -v amdgpu.ids | sed "s|^|$(basename $(dirname $L)) |" | cut -c1-140
done
