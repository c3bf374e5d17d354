#!/bin/bash
# Round 6: the 3D tracer after the convex-enclosure path (all 3D tests,
# interior L2 / L3 throughput with and without it, SQ counters at L3), the
# F_raw CSC boundary test and its C2 timing.
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_trace3d.py \
  "tests/test_gpu_boundary.py::test_F_csc_equals_host_transpose" > gpurun_out/r6/pytest_f.log 2>&1 || { tail -40 gpurun_out/r6/pytest_f.log; exit 1; }
tail -2 gpurun_out/r6/pytest_f.log
rm -f gpurun_out/r6/trace3d_interior.log
for L in 2 3; do
  timeout -k 10 200 python -u tools/bench_trace3d.py --interior --level $L --cpu-rows 2 >> gpurun_out/r6/trace3d_interior.log 2>&1 || { tail -20 gpurun_out/r6/trace3d_interior.log; exit 1; }
  RTHX_T3_NO_CVX=1 timeout -k 10 200 python -u tools/bench_trace3d.py --interior --level $L --cpu-rows 0 >> gpurun_out/r6/trace3d_interior.log 2>&1 || { tail -20 gpurun_out/r6/trace3d_interior.log; exit 1; }
done
grep config4 gpurun_out/r6/trace3d_interior.log | sed -e 's/BVH {.*convex_enclosure/convex_enclosure/'
timeout -k 10 300 python -u tools/host_boundary_cost.py --gpu > gpurun_out/r6/host_boundary_cost.log 2>&1 || { tail gpurun_out/r6/host_boundary_cost.log; exit 1; }
cat gpurun_out/r6/host_boundary_cost.log
bash tools/gpu_sq3d.sh interior_L3 --interior --level 3 > gpurun_out/r6/sq3d_interior_L3.txt 2>&1 || { tail -20 gpurun_out/r6/sq3d_interior_L3.txt; exit 1; }
grep -E "VALU |VMEM_RD|lane|wait" gpurun_out/r6/sq3d_interior_L3.txt
