#!/bin/bash
# C5 at 1e9 rays per band: the packed 16-bit histogram (82 KB of LDS, one
# 1024-lane workgroup per CU) against hash-tallied row parts small enough for
# two workgroups per CU (RTHX_FORCE_HASH + RTHX_HASH_MAX), trace + part merge.
export RTHX_DEV_KNOBS=1
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
L=raytraceheattransfer.jl_amd/csrc/_build/librthx.so
for b in 0 3; do
  timeout -k 10 300 python tools/ab.py --c5-bin $b --rays 1000000000 --rounds 3 --steps 2 \
    --sets="none|RTHX_FORCE_HASH=1:RTHX_HASH_MAX=8192|RTHX_FORCE_HASH=1:RTHX_HASH_MAX=4096|RTHX_TRACE_THREADS=512" $L >> $OUT/c5occ.log 2>&1 || { tail $OUT/c5occ.log; exit 1; }
done
grep -v amdgpu.ids $OUT/c5occ.log
