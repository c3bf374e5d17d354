#!/bin/bash
# Round 5: bench.py's fallback when pipelined steps fault (forced with
# RTHX_LB_WAIT_US=0: every look-back wait gives up), then a normal run.
set -o pipefail
mkdir -p gpurun_out
RTHX_DEV_KNOBS=1 RTHX_LB_WAIT_US=0 timeout -k 10 300 python bench.py --no-cpu --faithful-steps 0 --steps 10 --warmup 2 > gpurun_out/bench_fb.json 2> gpurun_out/bench_fb.err || { tail gpurun_out/bench_fb.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_fb.err | tail -2
python -c "
import json; d=json.loads(open('gpurun_out/bench_fb.json').read().strip().splitlines()[-1])
print('forced faults:', d['value'], d['step_mode'], d['steps_checked'], d['pipelined_step_faults'])"
timeout -k 10 300 python bench.py --no-cpu --faithful-steps 0 --steps 20 --warmup 5 > gpurun_out/bench_ok.json 2>/dev/null || exit 1
python -c "
import json; d=json.loads(open('gpurun_out/bench_ok.json').read().strip().splitlines()[-1])
print('normal:', d['value'], d['step_mode'], d['steps_checked'], d['pipelined_step_faults'])"
