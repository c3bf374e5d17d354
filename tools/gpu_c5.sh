#!/bin/bash
# C5 / multi-polygon iteration: parity tests, then C5 throughput at 1e8 and 1e9 rays per band.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_n.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_c5.log 2>&1 || { tail -40 gpurun_out/pytest_c5.log; exit 1; }
tail -2 gpurun_out/pytest_c5.log
timeout -k 10 200 python tools/bench_configs.py --only C5 > gpurun_out/configs_c5.log 2>&1 || { cat gpurun_out/configs_c5.log; exit 1; }
timeout -k 10 200 python tools/bench_configs.py --only C5 --rays 1e9 --steps 3 >> gpurun_out/configs_c5.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/configs_c5.log
if [ "${SQ:-0}" = "1" ]; then
  bash tools/gpu_sq_any.sh c5 trace_exchange_kernel 999956940 python3 $PWD/tools/bench_configs.py --only C5 --rays 1e9 --steps 1 --bins 0 --no-ramp > gpurun_out/sq_c5.log 2>&1 || exit 1
  grep -v "^  SQ_" gpurun_out/sq_c5.log
fi
