#!/bin/bash
# Rank-0 shard of the C2 job at emulated W under environment variants:
#   bash tools/gpu_split_env_ab.sh "W..." "MODE..." "ENV1;ENV2;..." [extra bench.py flags]   (ENV: space-separated VAR=VAL, or "-")
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
WS=${1:-"4 8"}
MODES=${2:-"strong weak"}
IFS=';' read -ra ENVS <<< "${3:--}"
EXTRA=${4:-}
for E in "${ENVS[@]}"; do
  for MODE in $MODES; do
    for W in $WS; do
      if [ $W = 1 ]; then extra=""; else extra="--emulate-world $W"; fi
      if [ $MODE = strong ]; then extra="$extra --strong"; fi
      envs=""; [ "$E" != "-" ] && envs="$E"
      env $envs timeout -k 10 120 python bench.py --no-cpu --faithful-steps 0 --steps 50 --warmup 10 $extra $EXTRA 2>>gpurun_out/split_env.err \
        | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
c = d['config']
print(f\"{'$E':>40s} $MODE W={$W}  rows {c['rays_per_step'] // c['rays_per_emitter']:6d}  R={c['rays_per_emitter']:6d}  \"
      f\"ms/step {d['ms_per_step']:.4f}  kernel {d['roofline']['avg_kernel_ms']:.4f}  pack {d['pack_ms']:.4f}  \"
      f\"rank-0 {(d.get('rank0_mrays_s') or d['value'])/1e3:.1f} Grays/s\", flush=True)
" || exit 1
    done
  done
done
