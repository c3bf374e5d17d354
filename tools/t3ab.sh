#!/bin/bash
# GPU box: 3D tracer parity tests, then config-4 throughput of the in-tree
# build beside variants (RTHX_LIB) -- bash tools/t3ab.sh [variant dir ...]
set -o pipefail
OUT=gpurun_out
CS=raytraceheattransfer.jl_amd/csrc
timeout -k 10 300 python -u -m pytest tests/test_gpu_trace3d.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/t3.log 2>&1 || { tail -30 $OUT/t3.log; exit 1; }
tail -1 $OUT/t3.log
for cfg in "--ndim 10 --level 3" "--ndim 20 --level 4"; do
  for v in "$@"; do
    RTHX_LIB=$CS/$v/librthx.so timeout -k 10 200 python tools/bench_trace3d.py $cfg --cpu-rows 0 2>&1 | grep config4 | sed "s|^|$v |" || exit 1
  done
  timeout -k 10 200 python tools/bench_trace3d.py $cfg --cpu-rows 0 2>&1 | grep config4 | sed 's/^/build /' || exit 1
  timeout -k 10 200 python tools/bench_trace3d.py $cfg --cpu-rows 0 --no-groups 2>&1 | grep config4 | sed 's/^/build /' || exit 1
done
