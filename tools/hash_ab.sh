#!/bin/bash
# A/B of the large-N hash tally knobs on L301 (301x301, N = 91805) at 1e8 and
# 9e8 rays: output by bitmap or sort, table cap, fill limit, workgroup size.
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
run() {
  echo "== $*" >> $OUT/hash_ab.log
  env "$@" timeout -k 10 120 python tools/bench_configs.py --only L301 $RAYS --steps 5 >> $OUT/hash_ab.log 2>&1 || exit 1
}
: > $OUT/hash_ab.log
RAYS=""
run X=0
run RTHX_HASH_SORT=1
run RTHX_TRACE_THREADS=256
run RTHX_HASH_LOAD_PCT=75
run RTHX_HASH_LOAD_PCT=75 RTHX_TRACE_THREADS=256
run RTHX_HASH_LOAD_PCT=30
RAYS="--rays 9e8"
run X=0
run RTHX_HASH_LOAD_PCT=75
run RTHX_HASH_MAX=4096
run RTHX_HASH_MAX=8192
grep -v amdgpu.ids $OUT/hash_ab.log
