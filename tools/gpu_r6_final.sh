#!/bin/bash
# Round 6 evidence refresh (from the repo root, on the GPU box): the GPU test
# suite (accuracy record), bench line + rocprof kernel stats + PMC traffic
# (gpu_profile.sh), headline SQ counters (gpu_sq.sh), the config table, C5
# at 1e9 rays per band, the 3D tracer (config 4 cube + sphere and interior),
# and smoke().
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
TAG=${1:-r6}
OUT=gpurun_out
mkdir -p $OUT
RTHX_ACCURACY_RECORD=$OUT/accuracy_$TAG.json timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu_$TAG.log 2>&1 || { tail -30 $OUT/pytest_gpu_$TAG.log; exit 1; }
tail -1 $OUT/pytest_gpu_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$TAG.log 2>&1 || { tail $OUT/smoke_$TAG.log; exit 1; }
tail -2 $OUT/smoke_$TAG.log
bash tools/gpu_profile.sh $TAG > $OUT/profile_$TAG.log 2>&1 || { tail -20 $OUT/profile_$TAG.log; exit 1; }
tail -c 400 $OUT/bench_$TAG.json
bash tools/gpu_sq.sh sq_$TAG > $OUT/sq_report_$TAG.txt 2>&1 || { tail $OUT/sq_report_$TAG.txt; exit 1; }
timeout -k 10 300 python tools/bench_configs.py > $OUT/configs_$TAG.log 2>&1 || { cat $OUT/configs_$TAG.log; exit 1; }
timeout -k 10 300 python tools/bench_configs.py --only C5 --rays 1e9 --steps 3 >> $OUT/configs_$TAG.log 2>&1 || exit 1
grep -v amdgpu.ids $OUT/configs_$TAG.log
for c in "11 3" "11 2" "20 4" "10 3"; do
  timeout -k 10 300 python tools/bench_trace3d.py --ndim ${c% *} --level ${c#* } >> $OUT/trace3d_$TAG.log 2>&1 || exit 1
done
for L in 2 3; do
  timeout -k 10 300 python tools/bench_trace3d.py --interior --level $L >> $OUT/trace3d_$TAG.log 2>&1 || exit 1
done
grep config4 $OUT/trace3d_$TAG.log | cut -c1-90,300-480
# the driver's multi-GPU launch shape rehearsed on this one GPU (2 ranks share
# device 0: a code-path check, no scaling claim)
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 2 --philox10-steps 0 --faithful-steps 0 > $OUT/bench2_$TAG.log 2>&1 || { tail -20 $OUT/bench2_$TAG.log; exit 1; }
grep '"metric"' $OUT/bench2_$TAG.log | cut -c1-200
