#!/bin/bash
# Round 6: the convex-enclosure fast path of the 3D tracer (icosphere seen
# from inside): its tests, then throughput at L2 / L3 with and without it.
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_trace3d.py \
  -k "convex" > gpurun_out/r6/pytest_t3.log 2>&1 || { tail -40 gpurun_out/r6/pytest_t3.log; exit 1; }
tail -3 gpurun_out/r6/pytest_t3.log
for L in 2 3; do
  timeout -k 10 200 python -u tools/bench_trace3d.py --interior --level $L --cpu-rows 0 >> gpurun_out/r6/trace3d_interior.log 2>&1 || { tail -20 gpurun_out/r6/trace3d_interior.log; exit 1; }
  RTHX_T3_NO_CVX=1 timeout -k 10 200 python -u tools/bench_trace3d.py --interior --level $L --cpu-rows 0 >> gpurun_out/r6/trace3d_interior.log 2>&1 || { tail -20 gpurun_out/r6/trace3d_interior.log; exit 1; }
done
cat gpurun_out/r6/trace3d_interior.log
bash tools/gpu_sq3d.sh interior_L3 --interior --level 3 > gpurun_out/r6/sq3d_interior_L3.txt 2>&1 || { tail -20 gpurun_out/r6/sq3d_interior_L3.txt; exit 1; }
cat gpurun_out/r6/sq3d_interior_L3.txt | tail -30
