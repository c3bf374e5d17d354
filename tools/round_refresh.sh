#!/bin/bash
# Round evidence refresh on the GPU box (from the repo root):
#   GPU test suite, bench line + rocprof stats + PMC traffic (gpu_profile.sh),
#   per-config throughput table and the config-4 3D tracer.
#   bash tools/round_refresh.sh [tag]
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
TAG=${1:-r1}
OUT=gpurun_out
mkdir -p $OUT
RTHX_ACCURACY_RECORD=$OUT/accuracy_$TAG.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/gpu_profile.sh $TAG || exit 1
timeout -k 10 300 python tools/bench_configs.py > $OUT/configs.log 2>&1 || { cat $OUT/configs.log; exit 1; }
timeout -k 10 300 python tools/bench_configs.py --only C5 --rays 1e9 --steps 3 >> $OUT/configs.log 2>&1 || exit 1
grep -v amdgpu.ids $OUT/configs.log
timeout -k 10 300 python tools/bench_trace3d.py --ndim 11 --level 3 > $OUT/trace3d.log 2>&1 || { cat $OUT/trace3d.log; exit 1; }
timeout -k 10 300 python tools/bench_trace3d.py --ndim 11 --level 2 --cpu-rows 0 >> $OUT/trace3d.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_trace3d.py --ndim 20 --level 4 --cpu-rows 0 >> $OUT/trace3d.log 2>&1 || exit 1
grep config4 $OUT/trace3d.log
