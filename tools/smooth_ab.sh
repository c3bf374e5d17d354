#!/bin/bash
# GPU box: smoothing/solve tests, then the C2 smoothing timing of the in-tree
# build beside variants (RTHX_LIB), then a rocprofv3 kernel-stats pass of the
# build -- bash tools/smooth_ab.sh [variant dir under csrc/ ...]
set -o pipefail
OUT=gpurun_out
CS=raytraceheattransfer.jl_amd/csrc
timeout -k 10 400 python -u -m pytest tests/test_gpu_smooth.py tests/test_gpu_solve.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/sm.log 2>&1 || { tail -30 $OUT/sm.log; exit 1; }
tail -1 $OUT/sm.log
for v in "$@"; do
  RTHX_LIB=$CS/$v/librthx.so timeout -k 10 300 python tools/bench_smooth.py --repeat 2 2>&1 | grep -E "smooth_F|row-sum" | sed "s|^|$v |" || exit 1
done
timeout -k 10 300 python tools/bench_smooth.py --repeat 2 2>&1 | grep -E "smooth_F|row-sum" | sed 's/^/build /' || exit 1
export TMPDIR=/tmp
R=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_smooth -o run -- python3 $R/tools/bench_smooth.py --repeat 1 > $R/$OUT/prof_smooth.log 2>&1 || exit 1
cd $R && python tools/pmc_summary.py stats $OUT/prof_smooth > $OUT/smooth_stats.json && python -c "
import json; d=json.load(open('$OUT/smooth_stats.json'))
for k in sorted(d['kernels'], key=lambda k: -k['total_ns'])[:10]: print('%-40s %6d calls  avg %9.1f us  total %8.2f ms' % (k['name'][:40], k['calls'], k['avg_ns']/1e3, k['total_ns']/1e6))"
