#!/bin/bash
# C5 / multi-polygon iteration on the GPU box (repo root):
#   bash tools/gpu_c5.sh TAG [SQ=1]
# 1. the 8-band C5 call at 1e9 rays per band (tools/bench_c5_bands.py),
# 2. the MLAT / multi-polygon parity tests (exact against the CPU restatement),
# 3. SQ=1: SQ counter passes of band 0 (the longest walks).
set -o pipefail
TAG=${1:-c5}
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_c5_bands.py --rays 1e9 --steps 2 > gpurun_out/c5b_$TAG.log 2>&1 || { cat gpurun_out/c5b_$TAG.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c5b_$TAG.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "multi_polygon or coarse_lds or c5 or split_part or spectral" --timeout 400 --timeout-method thread \
  > gpurun_out/pt_c5_$TAG.log 2>&1 || { tail -40 gpurun_out/pt_c5_$TAG.log; exit 1; }
tail -1 gpurun_out/pt_c5_$TAG.log
if [ "${SQ:-0}" = "1" ]; then
  bash tools/gpu_sq_any.sh c5b0_$TAG trace_exchange_kernel 999956940 python3 $PWD/tools/bench_configs.py --only C5 \
    --rays 1e9 --steps 1 --bins 0 --no-ramp > gpurun_out/sq_c5b0_$TAG.log 2>&1 || exit 1
  grep -v "^  SQ_[A-Z_]*  " gpurun_out/sq_c5b0_$TAG.log
  grep "SQ_INSTS_SALU\|SQ_INSTS_VALU \|SQ_INSTS_LDS" gpurun_out/sq_c5b0_$TAG.log
fi
