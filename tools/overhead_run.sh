#!/bin/bash
# fixed per-row cost (LDS zero + compaction) vs ray cost: bench at tiny R
for rays in 106050 1060500 10605000 100000000; do
  timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu --rays-per-gpu $rays 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('rays', $rays, 'R', d['config']['rays_per_emitter'], d['roofline']['avg_kernel_ms'], 'ms')" || exit 1
done
