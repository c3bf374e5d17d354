#!/bin/bash
# Round-4 evidence refresh (GPU box, repo root), in two calls:
#   bash tools/gpu_round3_final.sh TAG a   GPU tests, bench + rocprof stats + PMC
#                                          traffic, per-config table (C5 per band
#                                          and total), 3D tracer, mesh() pipeline,
#                                          SQ counters of the headline kernel
#   bash tools/gpu_round3_final.sh TAG b   SQ counters of C5 band 0, C5's 8-rank emulation, strong-scaling
#                                          emulation of C2, the direct-method cases
#                                          and D2's SQ counters, the 3D tracer's SQ
#                                          counters, smoke()
set -o pipefail
OUT=gpurun_out
TAG=${1:-r4}
PART=${2:-a}
mkdir -p $OUT
if [ "$PART" = a ]; then
  bash tools/round_refresh.sh $TAG || exit 1
  timeout -k 10 200 python tools/bench_configs.py --only L301 >> $OUT/configs.log 2>&1 || exit 1
  timeout -k 10 200 python tools/bench_pipeline.py --repeat 2 > $OUT/pipeline.log 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_c5_bands.py > $OUT/c5_bands.log 2>&1 || exit 1
  grep -v amdgpu $OUT/c5_bands.log
  bash tools/gpu_sq.sh $TAG > $OUT/sq_$TAG.log 2>&1 || exit 1
  grep -v "^  SQ_" $OUT/sq_$TAG.log
else
  bash tools/gpu_sq_any.sh c5b0_$TAG trace_exchange_kernel 999956940 python3 $PWD/tools/bench_configs.py --only C5 \
    --rays 1e9 --steps 1 --bins 0 --no-ramp > $OUT/sq_c5b0_$TAG.log 2>&1 || exit 1
  grep -v "^  SQ_" $OUT/sq_c5b0_$TAG.log
  timeout -k 10 300 python tools/bench_c5_bands.py --emulate-world 8 --rays 1e9 --steps 2 > $OUT/c5_emulated.log 2>&1 || exit 1
  grep -v amdgpu $OUT/c5_emulated.log
  bash tools/gpu_strong.sh > $OUT/strong_emulated.log 2>&1 || exit 1
  cat $OUT/strong_emulated.log
  timeout -k 10 300 python tools/bench_direct.py > $OUT/direct.log 2>&1 || exit 1
  grep -v amdgpu $OUT/direct.log
  bash tools/gpu_sq_direct.sh D2 > $OUT/sq_direct_D2_$TAG.log 2>&1 || exit 1
  grep -v "^  SQ_" $OUT/sq_direct_D2_$TAG.log
  bash tools/gpu_sq3d.sh sq3d_$TAG --ndim 11 --level 3 > $OUT/sq3d_$TAG.log 2>&1 || exit 1
  grep -v "^  SQ_" $OUT/sq3d_$TAG.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
fi
