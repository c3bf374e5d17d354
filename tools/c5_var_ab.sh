#!/bin/bash
# C5 A/B over librthx variants (csrc/_variants/<name>/librthx.so), 1e8 and 1e9 rays per band.
#   bash tools/c5_var_ab.sh name1 name2 ...   ("main" = csrc/_build)
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
: > $OUT/c5_var_ab.log
for v in "$@"; do
  if [ "$v" = main ]; then lib=$PWD/raytraceheattransfer.jl_amd/csrc/_build/librthx.so; else lib=$PWD/raytraceheattransfer.jl_amd/csrc/_variants/$v/librthx.so; fi
  for rays in 1e8 1e9; do
    echo "== $v $rays" >> $OUT/c5_var_ab.log
    RTHX_LIB=$lib timeout -k 10 120 python tools/bench_configs.py --only C5 --rays $rays --steps 4 --bins 0,4,7 >> $OUT/c5_var_ab.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $OUT/c5_var_ab.log
