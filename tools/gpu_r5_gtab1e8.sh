#!/bin/bash
# Round 5: C5 at 1e8 rays per band, LDS tables (csrc/_ab/gtab0) against the
# in-tree global tables, two rounds.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for v in "lds raytraceheattransfer.jl_amd/csrc/_ab/gtab0/librthx.so" "global raytraceheattransfer.jl_amd/csrc/_build/librthx.so"; do
    set -- $v
    RTHX_LIB=$2 timeout -k 10 300 python tools/bench_configs.py --only C5 --steps 3 > gpurun_out/c5_1e8_$1.log 2>&1 || { tail gpurun_out/c5_1e8_$1.log; exit 1; }
    echo "$1: $(grep 'band 0\|band 4\|total' gpurun_out/c5_1e8_$1.log | cut -c1-100 | tr '\n' '|')" | tee -a gpurun_out/gtab_1e8.log
  done
done
