#!/bin/bash
# Round 4: parity subset (with the async boundary test), wave-wide vs
# one-lane look-back A/B on the C2 rank-0 shards (blocking steps), the bench
# line pipelined and blocking, the CSR overflow cost.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_boundary.py tests/test_gpu_large_n.py tests/test_gpu_trace3d.py -m gpu -x -q \
  --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_c.log 2>&1 || { tail -40 gpurun_out/pt_c.log; exit 1; }
tail -n 1 gpurun_out/pt_c.log
LB0=RTHX_LIB=raytraceheattransfer.jl_amd/csrc/_ab/lb0/librthx.so
bash tools/gpu_split_env_ab.sh "1 8 4" "strong" "-;$LB0;-;$LB0" --blocking > gpurun_out/lb_ab.log 2>&1 || exit 1
bash tools/gpu_split_env_ab.sh "1 8 4 2" "strong" "-" > gpurun_out/async_strong.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 50 --warmup 20 > gpurun_out/bench_r4c.log 2>&1 || { tail -20 gpurun_out/bench_r4c.log; exit 1; }
tail -n 1 gpurun_out/bench_r4c.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 50 --warmup 20 --blocking --no-cpu --faithful-steps 0 > gpurun_out/bench_r4c_blocking.log 2>&1 || exit 1
timeout -k 10 120 python tools/overflow_cost.py > gpurun_out/overflow_cost.json 2>gpurun_out/overflow_cost.err || exit 1
cat gpurun_out/overflow_cost.json
