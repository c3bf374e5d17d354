#!/bin/bash
# C5 row tally A/B: packed histogram vs hash tables (cap variants), 1e8 and 1e9 rays per band.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/c5_tally_ab.log
for rays in 1e8 1e9; do
  for v in "X=0" "RTHX_FORCE_HASH=1" "RTHX_FORCE_HASH=1 RTHX_HASH_MAX=8192" "RTHX_FORCE_HASH=1 RTHX_HASH_MAX=4096" "RTHX_FORCE_HASH=1 RTHX_HASH_MAX=4096 RTHX_TRACE_THREADS=256"; do
    echo "== $rays $v" >> $OUT/c5_tally_ab.log
    env $v timeout -k 10 120 python tools/bench_configs.py --only C5 --rays $rays --steps 4 --bins 0,4,7 >> $OUT/c5_tally_ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $OUT/c5_tally_ab.log
