#!/bin/bash
# Round 4: wave-wide look-back x tail split A/B on the C2 rank-0 shards
# (parity subset first).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider -k "split or shard or lookback or c1 or c2 or c3 or edge" \
  > gpurun_out/pt_c.log 2>&1 || { tail -40 gpurun_out/pt_c.log; exit 1; }
tail -n 1 gpurun_out/pt_c.log
LB0=RTHX_LIB=raytraceheattransfer.jl_amd/csrc/_ab/lb0/librthx.so
bash tools/gpu_split_env_ab.sh "1 8 4" "strong" "-;RTHX_TAIL_SPLIT=1;$LB0;$LB0 RTHX_TAIL_SPLIT=1;RTHX_TAIL_SPLIT=2" > gpurun_out/lb_tail_ab.log 2>&1 || exit 1
