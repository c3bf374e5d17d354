#!/bin/bash
# Round 5 A/Bs in one call: (1) 2D emission Philox rounds 10 (in-tree) vs 7
# (csrc/_ab/p7) on the headline bench (timing only); (2) the box hull's
# interior bounding-ball skip (csrc/_ab/ball) vs the in-tree build on the
# config-4 3D scene, after the 3D GPU tests pass on the ball build.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out/r5
O=gpurun_out/r5
IN=raytraceheattransfer.jl_amd/csrc/_build/librthx.so
P7=raytraceheattransfer.jl_amd/csrc/_ab/p7/librthx.so
BALL=raytraceheattransfer.jl_amd/csrc/_ab/ball/librthx.so
RTHX_LIB=$BALL timeout -k 10 400 python -u -m pytest tests/test_gpu_trace3d.py -q -x --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_t3_ball.log 2>&1 || { tail -30 $O/pytest_t3_ball.log; exit 1; }
tail -1 $O/pytest_t3_ball.log
for r in 1 2; do
  for v in "base $IN" "ball $BALL"; do
    set -- $v
    for L in 3 4; do
      RTHX_LIB=$2 timeout -k 10 200 python tools/bench_trace3d.py --ndim 11 --level $L --cpu-rows 0 > $O/ab_$1_L${L}_$r.log 2>&1 || { tail $O/ab_$1_L${L}_$r.log; exit 1; }
      echo "$1 L$L: $(grep -o "kernel [0-9.]* ms ([0-9.]* Grays/s)" $O/ab_$1_L${L}_$r.log)" | tee -a $O/ab_ball.log
    done
  done
done
for r in 1 2 3; do
  for v in "philox10 $IN" "philox7 $P7"; do
    set -- $v
    RTHX_LIB=$2 timeout -k 10 200 python bench.py --no-cpu --faithful-steps 0 --steps 30 > $O/ab_$1_$r.json 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('$O/ab_$1_$r.json').read().strip().splitlines()[-1])
print('$1', 'value', d['value'], 'ms', d['ms_per_step'], 'kernel', d['roofline']['avg_kernel_ms'])" | tee -a $O/ab_philox.log
  done
done
