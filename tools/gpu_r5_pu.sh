#!/bin/bash
# Round 5: Philox blocks with their uniform first rounds on scalar
# instructions (philox_block_u) -- GPU parity (2D, 3D, direct), then A/B
# against the build before it (csrc/_ab/base) on C2, C5 bands 0 / 4 and the
# 3D config 4, and the headline SQ counters.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
IN=raytraceheattransfer.jl_amd/csrc/_build/librthx.so
B=raytraceheattransfer.jl_amd/csrc/_ab/base/librthx.so
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_trace3d.py tests/test_gpu_direct.py tests/test_gpu_boundary.py -m gpu -x -q \
  --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_pu.log 2>&1 || { tail -40 gpurun_out/pt_pu.log; exit 1; }
tail -1 gpurun_out/pt_pu.log
timeout -k 10 300 python tools/ab.py --rounds 10 $B $IN 2>&1 | grep -v amdgpu.ids | sed 's/^/C2  /' | tee gpurun_out/ab_pu.log || exit 1
bash tools/gpu_ab_c5.sh pu "0 4" $B $IN || exit 1
for r in 1 2; do
  for v in "base $B" "new $IN"; do
    set -- $v
    RTHX_LIB=$2 timeout -k 10 200 python tools/bench_trace3d.py --ndim 11 --level 3 --cpu-rows 0 > gpurun_out/t3_pu_$1.log 2>&1 || { tail gpurun_out/t3_pu_$1.log; exit 1; }
    echo "3D L3 $1: $(grep -o 'kernel [0-9.]* ms ([0-9.]* Grays/s)' gpurun_out/t3_pu_$1.log)" | tee -a gpurun_out/ab_pu.log
  done
done
bash tools/gpu_sq.sh sq_pu > gpurun_out/sq_report_pu.txt 2>&1 || { tail gpurun_out/sq_report_pu.txt; exit 1; }
grep "SQ_INSTS_VALU \|lane" gpurun_out/sq_report_pu.txt
