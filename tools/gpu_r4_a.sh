#!/bin/bash
# Round 4: split / workgroup-size A/B at the emulated W=8 strong shard and at
# W=1, then config 4 at the surveyed size (cube 11x11 + icosphere L2 / L3).
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_split_env_ab.sh "8" "strong" "RTHX_SPLIT_BELOW=1 RTHX_TRACE_THREADS=256;RTHX_SPLIT_BELOW=1 RTHX_TRACE_THREADS=512;RTHX_SPLIT_BELOW=1 RTHX_TRACE_THREADS=1024;RTHX_SPLIT_TARGET=2652 RTHX_TRACE_THREADS=256;RTHX_SPLIT_TARGET=3978 RTHX_TRACE_THREADS=256;RTHX_SPLIT_TARGET=2652 RTHX_TRACE_THREADS=1024" > gpurun_out/ab_w8b.log 2>&1 || exit 1
bash tools/gpu_split_env_ab.sh "1" "weak" "-;RTHX_TRACE_THREADS=256;RTHX_SPLIT_BELOW=100000 RTHX_SPLIT_TARGET=21210;RTHX_SPLIT_BELOW=100000 RTHX_SPLIT_TARGET=21210 RTHX_NO_LOOKBACK=1" >> gpurun_out/ab_w8b.log 2>&1 || exit 1
for nl in "11 2" "11 3" "10 3" "20 4"; do
  set -- $nl
  timeout -k 10 200 python tools/bench_trace3d.py --ndim $1 --level $2 --cpu-rows 0 >> gpurun_out/trace3d_r4.log 2>&1 || exit 1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_trace3d.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k config4 > gpurun_out/pt_config4.log 2>&1
