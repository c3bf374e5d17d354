#!/bin/bash
# Round 5: two-pass box-hull 3D tracer -- tests, hull vs plain walk on
# config 4, SQ counters of both at cube 11x11 + L3.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out/r5
O=gpurun_out/r5
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_trace3d.py > $O/pt_t3d.log 2>&1; rc=$?
tail -n 5 $O/pt_t3d.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for c in "11 3" "20 4" "11 2"; do
    nd=${c% *}; lv=${c#* }
    for v in "hull 0" "walk 1"; do
      set -- $v
      RTHX_T3_NO_HULL=$2 timeout -k 10 200 python tools/bench_trace3d.py --ndim $nd --level $lv --cpu-rows 0 2>&1 \
        | grep config4 | sed "s|^|$1 |" >> $O/t3_hull_ab3.log || exit 1
    done
  done
done
cut -c1-60,300-420 $O/t3_hull_ab3.log
RTHX_T3_NO_HULL=0 bash tools/gpu_sq3d.sh hull3 --ndim 11 --level 3 > $O/sq3d_hull3.txt 2>&1 || { tail $O/sq3d_hull3.txt; exit 1; }
cp gpurun_out/sq_hull3.json $O/
tail -n 30 $O/sq3d_hull3.txt
