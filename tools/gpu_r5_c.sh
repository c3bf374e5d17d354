#!/bin/bash
# Round 5: box-hull 3D tracer -- tests, then A/B of the in-tree build (hull
# kernels at 6 waves), the 5-wave variant and the plain walk (RTHX_T3_NO_HULL=1).
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out/r5
O=gpurun_out/r5
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_trace3d.py > $O/pt_t3b.log 2>&1; rc=$?
tail -n 5 $O/pt_t3b.log
[ $rc -eq 0 ] || exit $rc
IN=raytraceheattransfer.jl_amd/csrc/_build/librthx.so
H5=raytraceheattransfer.jl_amd/csrc/_ab/h5/librthx.so
for r in 1 2; do
  for c in "11 3" "20 4" "11 2"; do
    nd=${c% *}; lv=${c#* }
    for v in "hull6 $IN 0" "hull5 $H5 0" "walk $IN 1"; do
      set -- $v
      RTHX_T3_NO_HULL=$3 RTHX_LIB=$2 timeout -k 10 200 python tools/bench_trace3d.py --ndim $nd --level $lv --cpu-rows 0 2>&1 \
        | grep config4 | sed "s|^|$1 |" >> $O/t3_hull_ab.log || exit 1
    done
  done
done
cut -c1-80,300-420 $O/t3_hull_ab.log
timeout -k 10 400 python tools/c5_assembly.py > $O/c5_assembly.log 2>&1 || { tail -20 $O/c5_assembly.log; exit 1; }
grep -v amdgpu.ids $O/c5_assembly.log
