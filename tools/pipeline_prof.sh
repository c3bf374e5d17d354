#!/bin/bash
# GPU box: whole C2 pipeline (trace -> smooth -> solve) timing and its
# rocprofv3 kernel statistics -- bash tools/pipeline_prof.sh
set -o pipefail
OUT=gpurun_out
R=$(pwd)
timeout -k 10 300 python tools/bench_pipeline.py 2>&1 | grep -v amdgpu.ids > $OUT/pipeline.log || exit 1
cat $OUT/pipeline.log
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_pipe -o run -- python3 $R/tools/bench_pipeline.py --repeat 1 > $R/$OUT/prof_pipe.log 2>&1 || exit 1
cd $R && python tools/pmc_summary.py stats $OUT/prof_pipe > $OUT/pipe_stats.json && python -c "
import json; d=json.load(open('$OUT/pipe_stats.json'))
for k in sorted(d['kernels'], key=lambda k: -k['total_ns'])[:16]: print('%-44s %6d calls  avg %9.1f us  total %8.2f ms' % (k['name'][:44], k['calls'], k['avg_ns']/1e3, k['total_ns']/1e6))"
