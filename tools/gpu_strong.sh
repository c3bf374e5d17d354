#!/bin/bash
# Strong-scaling diagnostic on one GPU (no scaling claim): rank 0's shard of a
# fixed 1e8-ray C2 job split over W = 1, 2, 4, 8 GPUs (bench.py --strong
# --emulate-world W: rows g = 0, W, 2W, ... with R = 1e8 / N rays each).
#   bash tools/gpu_strong.sh > gpurun_out/strong_emulated.log
set -o pipefail
for W in 1 2 4 8; do
  if [ $W = 1 ]; then extra=""; else extra="--emulate-world $W"; fi
  timeout -k 10 120 python bench.py --strong --no-cpu --faithful-steps 0 --steps 50 --warmup 10 $extra 2>/dev/null \
    | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
c = d['config']
print(f\"W={$W}  rank-0 rows {c['rays_per_step'] // c['rays_per_emitter']:6d}  R={c['rays_per_emitter']}  \"
      f\"ms/step {d['ms_per_step']:.4f} (blocking {d['blocking_ms_per_step']:.4f})  kernel {d['roofline']['avg_kernel_ms']:.4f} ms  pack {d['pack_ms']:.4f} ms  \"
      f\"rank-0 {d.get('rank0_mrays_s') or d['value']:.1f} Mrays/s\")
" || exit 1
done
