#!/bin/bash
# GPU test suite on the in-tree build, then the default bench line.
#   bash tools/gpu_check.sh TAG
set -o pipefail
TAG=${1:-chk}
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/pt_$TAG.log 2>&1 || { tail -40 gpurun_out/pt_$TAG.log; exit 1; }
tail -n 1 gpurun_out/pt_$TAG.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "
import json; d = json.loads(open('gpurun_out/bench_$TAG.json').read().strip().splitlines()[-1])
print('value', d['value'], 'ms/step', d['ms_per_step'], 'kernel', d['roofline']['avg_kernel_ms'], 'valu frac', d.get('roofline_valu', {}).get('frac'), 'faithful', d.get('faithful_sampling'))"
