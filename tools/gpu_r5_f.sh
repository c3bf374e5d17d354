#!/bin/bash
# Round 5: A/B of the 2D emission's Philox rounds (10, in-tree; 7, csrc/_ab/p7)
# on the headline bench (timing only: the p7 build's draws differ from the
# oracle's, so its counts are not checked here).
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out/r5
O=gpurun_out/r5
IN=raytraceheattransfer.jl_amd/csrc/_build/librthx.so
P7=raytraceheattransfer.jl_amd/csrc/_ab/p7/librthx.so
for r in 1 2 3; do
  for v in "philox10 $IN" "philox7 $P7"; do
    set -- $v
    RTHX_LIB=$2 timeout -k 10 200 python bench.py --no-cpu --faithful-steps 0 --steps 30 > $O/ab_$1_$r.json 2>/dev/null || exit 1
    python -c "
import json; d=json.loads(open('$O/ab_$1_$r.json').read().strip().splitlines()[-1])
print('$1', 'value', d['value'], 'ms', d['ms_per_step'], 'kernel', d['roofline']['avg_kernel_ms'])" | tee -a $O/ab_philox.log
  done
done
