#!/bin/bash
# Round 6: the convex-enclosure fast path of the 3D tracer (icosphere seen
# from inside): exactness tests, throughput at L2/L3 with and without it;
# then the band pipeline / accuracy / philox10 / bench script.
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_trace3d.py \
  > gpurun_out/r6/pytest_t3.log 2>&1 || { tail -40 gpurun_out/r6/pytest_t3.log; exit 1; }
tail -3 gpurun_out/r6/pytest_t3.log
for L in 2 3; do
  timeout -k 10 300 python -u tools/bench_trace3d.py --interior --level $L --cpu-rows 2 >> gpurun_out/r6/trace3d_interior.log 2>&1 || { tail -20 gpurun_out/r6/trace3d_interior.log; exit 1; }
  RTHX_T3_NO_CVX=1 timeout -k 10 300 python -u tools/bench_trace3d.py --interior --level $L --cpu-rows 0 >> gpurun_out/r6/trace3d_interior.log 2>&1 || { tail -20 gpurun_out/r6/trace3d_interior.log; exit 1; }
done
cat gpurun_out/r6/trace3d_interior.log
bash tools/gpu_r6_b.sh
