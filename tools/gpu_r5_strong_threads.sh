#!/bin/bash
# Round 5: the emulated strong shards with the workgroup size forced
# (RTHX_TRACE_THREADS 256 / 512 / 1024) against the occupancy choice.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
for t in auto 256 512 1024; do
  echo "== threads $t" >> gpurun_out/strong_threads.log
  if [ $t = auto ]; then
    timeout -k 10 400 bash tools/gpu_strong.sh >> gpurun_out/strong_threads.log 2>&1 || exit 1
  else
    RTHX_TRACE_THREADS=$t timeout -k 10 400 bash tools/gpu_strong.sh >> gpurun_out/strong_threads.log 2>&1 || exit 1
  fi
done
cat gpurun_out/strong_threads.log | cut -c1-110
