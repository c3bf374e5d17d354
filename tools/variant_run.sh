#!/bin/bash
# time bench.py against csrc/_variants/<name>/librthx.so for each name (interleaved twice)
for pass in 1 2; do
for m in "$@"; do
  RTHX_LIB=raytraceheattransfer.jl_amd/csrc/_variants/$m/librthx.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu $BENCH_ARGS 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('variant $m', d['roofline']['avg_kernel_ms'], 'ms', d['value'], 'Mray/s')" || exit 1
done
done
