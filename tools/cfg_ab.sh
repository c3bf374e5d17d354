#!/bin/bash
# Throughput A/B over librthx variants (csrc/_variants/<name>/librthx.so; "main" = csrc/_build).
#   ONLY=C2,C5 RAYS="1e8 1e9" BINS=0,4,7 bash tools/cfg_ab.sh name1 name2 ...
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
LOG=$OUT/cfg_ab.log
: > $LOG
for rays in ${RAYS:-1e8}; do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=$PWD/raytraceheattransfer.jl_amd/csrc/_build/librthx.so; else lib=$PWD/raytraceheattransfer.jl_amd/csrc/_variants/$v/librthx.so; fi
    echo "== $v $rays" >> $LOG
    RTHX_LIB=$lib timeout -k 10 150 python tools/bench_configs.py --only ${ONLY:-C2} --rays $rays --steps ${STEPS:-6} --bins ${BINS:-0,4,7} >> $LOG 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $LOG
