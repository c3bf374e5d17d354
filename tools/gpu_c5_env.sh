#!/bin/bash
# C5 bands under environment variants (one process per variant):
#   bash tools/gpu_c5_env.sh TAG "BINS" RAYS "ENV1" "ENV2" ...   ("-" = defaults)
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
TAG=$1; BINS=$2; RAYS=$3; shift 3
mkdir -p gpurun_out
for v in "$@"; do
  envs=""; [ "$v" != "-" ] && envs="$v"
  echo "== $v" | tee -a gpurun_out/c5env_$TAG.log
  env $envs timeout -k 10 240 python tools/bench_configs.py --only C5 --bins "$BINS" --rays $RAYS --steps 2 --no-ramp 2>&1 \
    | grep -v amdgpu.ids | tee -a gpurun_out/c5env_$TAG.log || exit 1
done
