#!/bin/bash
# run bench.py against each ablated library (diagnostic timings only)
for m in "$@"; do
  RTHX_LIB=raytraceheattransfer.jl_amd/csrc/_ablate/$m/librthx.so timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('mask $m', d['roofline']['avg_kernel_ms'], 'ms', d['value'], 'Mray/s')" || exit 1
done
