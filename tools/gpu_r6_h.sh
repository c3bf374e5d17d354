#!/bin/bash
# Round 6: deferred walks in the 3D fast-path kernels -- exactness (all 3D
# tests), then A/B against the same build without deferral (RTHX_T3_DEFER=0)
# on config 4 (cube + icosphere) and the icosphere seen from inside.
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_trace3d.py \
  tests/test_gpu_known_answers.py -k "3d or trace or icosphere or hull or convex or box" > gpurun_out/r6/pytest_h.log 2>&1 || { tail -40 gpurun_out/r6/pytest_h.log; exit 1; }
tail -2 gpurun_out/r6/pytest_h.log
L=raytraceheattransfer.jl_amd/csrc
rm -f gpurun_out/r6/defer_ab.log
for r in 1 2; do
  for lib in $L/_build/librthx.so $L/_ab/nodefer/librthx.so; do
    for c in "--ndim 11 --level 3" "--ndim 11 --level 2" "--ndim 20 --level 4" "--interior --level 2" "--interior --level 3"; do
      RTHX_LIB=$lib timeout -k 10 200 python tools/bench_trace3d.py $c --cpu-rows 0 2>&1 | grep config4 \
        | sed -e "s|^|$(basename $(dirname $lib)) |; s/BVH {.*}  kernel/kernel/" | cut -c1-200 >> gpurun_out/r6/defer_ab.log || exit 1
    done
  done
done
cat gpurun_out/r6/defer_ab.log
