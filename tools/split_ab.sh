#!/bin/bash
# GPU box: rank-0 shard timings of W-GPU jobs (bench.py --emulate-world) for
# the build and variants -- bash tools/split_ab.sh [variant dir under csrc/ ...]
set -o pipefail
CS=raytraceheattransfer.jl_amd/csrc
for v in build "$@"; do
  for w in 1 2 4 8; do
    EW=""; [ $w -gt 1 ] && EW="--emulate-world $w"
    if [ "$v" = build ]; then unset RTHX_LIB; else export RTHX_LIB=$CS/$v/librthx.so; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu $EW 2>/dev/null > gpurun_out/sab.json || exit 1
    python3 -c "
import json; d=json.load(open('gpurun_out/sab.json')); v=d['value'] or d['rank0_mrays_s']
print('%-14s W=%d %8.1f Grays/s per GPU  %.4f ms/step  trace %.4f ms' % ('$v', $w, v/1e3, d['ms_per_step'], d['roofline']['avg_kernel_ms']))"
  done
done
