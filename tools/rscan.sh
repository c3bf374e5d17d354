#!/bin/bash
# Trace time vs rays per emitter on the BASELINE domain (fixed per-launch
# cost = intercept of time vs rays).  Usage: tools/rscan.sh [lib]
LIBARG=${1:+RTHX_LIB=$1}
for rays in 1060500 10605000 50000000 100000000 200000000 400000000; do
  env $LIBARG timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --rays-per-gpu $rays 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rays', d['config']['rays_per_step'], 'R', d['config']['rays_per_emitter'], 'kernel_ms', d['roofline']['avg_kernel_ms'], 'step_ms', d['ms_per_step'])" || exit 1
done
