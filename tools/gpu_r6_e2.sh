#!/bin/bash
# Round 6: convex-enclosure fast path -- exactness, then the largest half-arc
# (RTHX_T3_CVX_ARC; auto = sqrt(1 - (r_in/r_out)^2) / 2) x the cube map's
# resolution (RTHX_T3_CVX_RES) at L2 / L3.
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_trace3d.py \
  -k "convex" > gpurun_out/r6/pytest_t3e2.log 2>&1 || { tail -40 gpurun_out/r6/pytest_t3e2.log; exit 1; }
tail -2 gpurun_out/r6/pytest_t3e2.log
for L in 2 3; do
  for arc in auto 0.02 0.04 0.08; do
    for res in 3 4; do
      if [ $arc = auto ]; then unset RTHX_T3_CVX_ARC; else export RTHX_T3_CVX_ARC=$arc; fi
      r=$(RTHX_T3_CVX_RES=$res timeout -k 10 200 python -u tools/bench_trace3d.py --interior --level $L --cpu-rows 0 2>/dev/null | grep config4) || exit 1
      echo "L$L arc $arc res $res: $(echo $r | sed -e 's/.*kernel/kernel/')" >> gpurun_out/r6/cvx_arc.log
    done
  done
done
cat gpurun_out/r6/cvx_arc.log
