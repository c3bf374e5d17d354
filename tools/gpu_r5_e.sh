#!/bin/bash
# Round 5: the hull's skip of a quad's second triangle -- tests, then A/B
# against the previous build (csrc/_ab/base) on config 4.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out/r5
O=gpurun_out/r5
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_trace3d.py > $O/pt_t3e.log 2>&1; rc=$?
tail -n 5 $O/pt_t3e.log
[ $rc -eq 0 ] || exit $rc
IN=raytraceheattransfer.jl_amd/csrc/_build/librthx.so
B=raytraceheattransfer.jl_amd/csrc/_ab/base/librthx.so
for r in 1 2; do
  for c in "11 3" "20 4" "11 2"; do
    nd=${c% *}; lv=${c#* }
    for v in "skipB $IN" "base $B"; do
      set -- $v
      RTHX_LIB=$2 timeout -k 10 200 python tools/bench_trace3d.py --ndim $nd --level $lv --cpu-rows 0 2>&1 \
        | grep config4 | sed "s|^|$1 |" >> $O/t3_skipb_ab.log || exit 1
    done
  done
done
cut -c1-60,300-420 $O/t3_skipb_ab.log
for L in 2 3; do
  timeout -k 10 120 python tools/bench_trace3d.py --interior --level $L --cpu-rows 0 >> $O/t3_interior2.log 2>&1 || exit 1
done
grep config4 $O/t3_interior2.log | cut -c1-60,250-420
