#!/bin/bash
# Round 5: the 3D tracer's box-hull fast path -- its tests, the whole 3D test
# file, then config 4 rates with and without the hull (RTHX_T3_NO_HULL=1).
set -o pipefail
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
mkdir -p gpurun_out/r5
O=gpurun_out/r5
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_trace3d.py > $O/pt_t3.log 2>&1; rc=$?
tail -n 40 $O/pt_t3.log
[ $rc -eq 0 ] || exit $rc
for H in 0 1; do
  export RTHX_T3_NO_HULL=$H
  timeout -k 10 120 python tools/bench_trace3d.py --ndim 11 --level 3 --cpu-rows 0 >> $O/t3_hull.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_trace3d.py --ndim 11 --level 2 --cpu-rows 0 >> $O/t3_hull.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_trace3d.py --ndim 20 --level 4 --cpu-rows 0 >> $O/t3_hull.log 2>&1 || exit 1
  timeout -k 10 120 python tools/bench_trace3d.py --ndim 10 --level 3 --cpu-rows 0 >> $O/t3_hull.log 2>&1 || exit 1
  echo "-- RTHX_T3_NO_HULL=$H done" >> $O/t3_hull.log
done
grep -v amdgpu.ids $O/t3_hull.log
