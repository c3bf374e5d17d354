#!/bin/bash
# Round 4: full GPU test suite, the default bench line, the tail-split A/B on
# the C2 rank-0 shards, and the 3D dynamic-top A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pytest_gpu_r4b.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_r4b.log; exit 1; }
tail -n 1 gpurun_out/pytest_gpu_r4b.log
timeout -k 10 300 python bench.py --steps 50 --warmup 20 > gpurun_out/bench_r4b.log 2>&1 || { tail -20 gpurun_out/bench_r4b.log; exit 1; }
tail -n 1 gpurun_out/bench_r4b.log | cut -c1-400
bash tools/gpu_split_env_ab.sh "1 8 4" "strong" "RTHX_TAIL_SPLIT=1;-;RTHX_TAIL_SPLIT=2;RTHX_TAIL_PCT=200" > gpurun_out/tail_ab_b.log 2>&1 || exit 1
bash tools/gpu_t3_dyn.sh b "- t3_512 t3_1024" "-;RTHX_T3_DYNTOP=1 RTHX_T3_BFS_TOP=8192" || exit 1
