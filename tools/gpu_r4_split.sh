#!/bin/bash
# Round 4: split-by-slots rule -- parity subset, then the C2 rank-0 shard at
# emulated W = 1..8 (strong: 1e8 rays per job; weak: 1e8 per GPU) and the
# one-GPU C5 projection at W = 8.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py tests/test_gpu_large_n.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "split or shard or lookback or c1 or large" \
  > gpurun_out/pt_split_r4.log 2>&1 || { tail -40 gpurun_out/pt_split_r4.log; exit 1; }
tail -n 1 gpurun_out/pt_split_r4.log
bash tools/gpu_split_env_ab.sh "1 2 4 8" "strong weak" "-" > gpurun_out/split_r4.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_c5_bands.py --emulate-world 8 --rays 1e9 --steps 2 > gpurun_out/c5_emulated_r4.log 2>&1 || exit 1
