#!/bin/bash
# Round 4: full GPU test suite, the default bench line, the tail-split A/B on
# the C2 rank-0 shards, the four-child 3D walk (parity, A/B), the direct
# method at 5 waves.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu_r4b.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r4b.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu_r4b.log
timeout -k 10 300 python bench.py --steps 50 --warmup 20 > gpurun_out/bench_r4b.log 2>&1 || { tail -20 gpurun_out/bench_r4b.log; exit 1; }
tail -n 1 gpurun_out/bench_r4b.log | cut -c1-400
bash tools/gpu_split_env_ab.sh "1 8 4" "strong" "RTHX_TAIL_SPLIT=1;-;RTHX_TAIL_SPLIT=2;RTHX_TAIL_PCT=200" > gpurun_out/tail_ab_b.log 2>&1 || exit 1
RTHX_T3_BVH4=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_trace3d.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pt_t3w4.log 2>&1 || { tail -30 gpurun_out/pt_t3w4.log; exit 1; }
tail -n 1 gpurun_out/pt_t3w4.log
bash tools/gpu_t3_dyn.sh b "-" "-;RTHX_T3_BVH4=1;RTHX_T3_BVH4=1 RTHX_T3_W4_THREADS=512;RTHX_T3_BVH4=1 RTHX_T3_W4_THREADS=256;RTHX_T3_DYNTOP=1 RTHX_T3_BFS_TOP=8192" || exit 1
bash tools/gpu_t3_dyn.sh b1024 "t3_1024" "RTHX_T3_DYNTOP=1 RTHX_T3_BFS_TOP=8192" || exit 1
bash tools/gpu_r4_d.sh || exit 1
