#!/bin/bash
# Round 5: the layered walk's x-wall segment resolved by x_wall_segment
# instead of layer_segment -- MLAT / C5 parity, then C5 bands 0 / 4 at 1e9
# rays against the build before it (csrc/_ab/base).
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
IN=raytraceheattransfer.jl_amd/csrc/_build/librthx.so
B=raytraceheattransfer.jl_amd/csrc/_ab/base/librthx.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -k "multi_polygon or coarse_lds or c5 or split_part or spectral or layer or wedges" --timeout 400 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pt_xwall.log 2>&1 || { tail -40 gpurun_out/pt_xwall.log; exit 1; }
tail -1 gpurun_out/pt_xwall.log
bash tools/gpu_ab_c5.sh xwall "0 4" $B $IN || exit 1
timeout -k 10 300 python tools/bench_configs.py --only C5 --rays 1e9 --steps 3 > gpurun_out/c5_xwall.log 2>&1 || exit 1
grep total gpurun_out/c5_xwall.log
