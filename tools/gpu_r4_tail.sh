#!/bin/bash
# Round 4: tail split (the last round of rows in parts) -- parity subset, then
# A/B of its parts and rows on the C2 rank-0 shard at emulated W = 1, 2, 4, 8.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py tests/test_gpu_large_n.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "split or shard or lookback or c1 or large or c2 or c3" \
  > gpurun_out/pt_tail.log 2>&1 || { tail -40 gpurun_out/pt_tail.log; exit 1; }
tail -n 1 gpurun_out/pt_tail.log
bash tools/gpu_split_env_ab.sh "1 8 4 2" "strong" "RTHX_TAIL_SPLIT=1;-;RTHX_TAIL_SPLIT=2;RTHX_TAIL_PCT=50;RTHX_TAIL_PCT=200" > gpurun_out/tail_ab.log 2>&1 || exit 1
bash tools/gpu_split_env_ab.sh "8" "weak" "RTHX_TAIL_SPLIT=1;-" >> gpurun_out/tail_ab.log 2>&1 || exit 1
