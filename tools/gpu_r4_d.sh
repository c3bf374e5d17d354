#!/bin/bash
# Round 4: direct method at 5 waves per SIMD (A/B), 3D dynamic top A/B.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_direct_ab.sh r4 D1,D2,D3 "" raytraceheattransfer.jl_amd/csrc/_build/librthx.so raytraceheattransfer.jl_amd/csrc/_ab/dw5/librthx.so || exit 1
timeout -k 10 120 python tools/overflow_cost.py > gpurun_out/overflow_cost.json 2>gpurun_out/overflow_cost.err || exit 1
