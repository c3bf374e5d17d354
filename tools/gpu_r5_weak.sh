#!/bin/bash
# Round 5: rank 0's shard of the weak-scaling job (1e8 rays per GPU, rows
# g = 0, W, 2W, ... with R = W * 1e8 / N) emulated on one GPU for W = 1..8
# (bench.py --emulate-world W; no scaling claim: one GPU).
set -o pipefail
mkdir -p gpurun_out
for W in 1 2 4 8; do
  if [ $W = 1 ]; then extra=""; else extra="--emulate-world $W"; fi
  timeout -k 10 200 python bench.py --no-cpu --faithful-steps 0 --steps 20 --warmup 5 $extra 2>/dev/null | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
c = d['config']
print(f\"weak W=$W  rank-0 rows {c['rays_per_step'] // c['rays_per_emitter']:6d}  R={c['rays_per_emitter']}  ms/step {d['ms_per_step']:.4f}  kernel {d['roofline']['avg_kernel_ms']:.4f} ms  rank-0 {d.get('rank0_mrays_s') or d['value']:.1f} Mrays/s\")
" | tee -a gpurun_out/weak_emulated.log || exit 1
done
