#!/bin/bash
# Round 6: convex-enclosure fast path -- exactness, then the cube map's
# resolution (RTHX_T3_CVX_RES cells per triangle edge) at L2 / L3.
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_trace3d.py \
  -k "convex" > gpurun_out/r6/pytest_t3e.log 2>&1 || { tail -40 gpurun_out/r6/pytest_t3e.log; exit 1; }
tail -2 gpurun_out/r6/pytest_t3e.log
for L in 2 3; do
  for res in 2 3 4 6; do
    echo "RTHX_T3_CVX_RES=$res" >> gpurun_out/r6/cvx_res.log
    RTHX_T3_CVX_RES=$res timeout -k 10 200 python -u tools/bench_trace3d.py --interior --level $L --cpu-rows 0 2>/dev/null | grep config4 >> gpurun_out/r6/cvx_res.log || exit 1
  done
done
sed -e 's/BVH {.*convex_enclosure/convex_enclosure/' gpurun_out/r6/cvx_res.log
