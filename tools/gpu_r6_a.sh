#!/bin/bash
# Round 6 first GPU call: the split-row hand-off's release/acquire fences
# (A/B against the round-5 library without them) and the emulated strong
# shards with rows split to RTHX_SPLIT_TARGET parts-slots; then the split and
# C2 parity tests.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out/r6
L=raytraceheattransfer.jl_amd/csrc
for W in 8 4; do
  echo "== strong W=$W" >> gpurun_out/r6/split_ab.log
  timeout -k 10 300 python tools/ab.py --stride $W --rounds 6 --steps 10 --env RTHX_SPLIT_TARGET=auto,2652,3978,5304,7956 \
    $L/_build/librthx.so $L/_ab/nofence/librthx.so >> gpurun_out/r6/split_ab.log 2>&1 || { tail gpurun_out/r6/split_ab.log; exit 1; }
done
cat gpurun_out/r6/split_ab.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_boundary.py \
  > gpurun_out/r6/pytest_a.log 2>&1; rc=$?
tail -5 gpurun_out/r6/pytest_a.log
exit $rc
