#!/bin/bash
# Round-2 evidence refresh (GPU box, repo root): GPU tests, bench + rocprof
# stats + PMC traffic, configs, 3D, pipeline, C5 bands, SQ of the headline.
set -o pipefail
OUT=gpurun_out
TAG=${1:-r2b}
bash tools/round_refresh.sh $TAG || exit 1
timeout -k 10 200 python tools/bench_configs.py --only L301 >> $OUT/configs.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_pipeline.py --repeat 2 > $OUT/pipeline.log 2>&1 || exit 1
grep -v amdgpu $OUT/pipeline.log
timeout -k 10 300 python tools/bench_c5_bands.py > $OUT/c5_bands.log 2>&1 || exit 1
grep -v amdgpu $OUT/c5_bands.log
bash tools/gpu_sq.sh $TAG > $OUT/sq_$TAG.log 2>&1 || exit 1
grep -v "^  SQ_" $OUT/sq_$TAG.log
