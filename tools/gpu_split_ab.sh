#!/bin/bash
# Split-row hand-off: parity tests, then rank-0 shards of the strong (1e8 rays
# per job) and weak (1e8 rays per GPU) C2 jobs at emulated W = 1..8, under
# the split settings given as "BELOW:TARGET" pairs.
#   bash tools/gpu_split_ab.sh TAG "2048:4096 4096:4096 4096:8192"
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
TAG=${1:-split}
SETS=${2:-"2048:4096"}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "split or shard or lookback or c1" \
  > gpurun_out/pt_$TAG.log 2>&1 || { tail -40 gpurun_out/pt_$TAG.log; exit 1; }
tail -n 1 gpurun_out/pt_$TAG.log
for S in $SETS; do
  export RTHX_SPLIT_BELOW=${S%%:*} RTHX_SPLIT_TARGET=${S##*:}
  for MODE in strong weak; do
    for W in 1 2 4 8; do
      if [ $W = 1 ]; then extra=""; else extra="--emulate-world $W"; fi
      if [ $MODE = strong ]; then extra="$extra --strong"; fi
      timeout -k 10 120 python bench.py --no-cpu --faithful-steps 0 --steps 50 --warmup 10 $extra 2>>gpurun_out/split_$TAG.err \
        | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
c = d['config']
print(f\"split {'$S':>10s} $MODE W={$W}  rows {c['rays_per_step'] // c['rays_per_emitter']:6d}  R={c['rays_per_emitter']:6d}  \"
      f\"ms/step {d['ms_per_step']:.4f}  kernel {d['roofline']['avg_kernel_ms']:.4f}  pack {d['pack_ms']:.4f}  \"
      f\"rank-0 {d.get('rank0_mrays_s') or d['value']:.1f} Mrays/s\", flush=True)
" || exit 1
    done
  done
done
if [ "${C5:-0}" = "1" ]; then
  timeout -k 10 300 python tools/bench_c5_bands.py --emulate-world 8 --rays 1e9 --steps 2 2>&1 | grep -v amdgpu.ids
fi
