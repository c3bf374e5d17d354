#!/bin/bash
# Round 5: cos / log tables from global memory (RTHX_GTAB=1, csrc/_ab/gtab)
# against the in-tree build (LDS tables): parity on the variant, then C2 / C3
# kernels, C5 bands 0 and 4, and the emulated strong shards.
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
mkdir -p gpurun_out
IN=raytraceheattransfer.jl_amd/csrc/_build/librthx.so
GT=raytraceheattransfer.jl_amd/csrc/_ab/gtab/librthx.so
RTHX_LIB=$GT timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 400 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/pt_gtab.log 2>&1 || { tail -40 gpurun_out/pt_gtab.log; exit 1; }
tail -1 gpurun_out/pt_gtab.log
timeout -k 10 300 python tools/ab.py --rounds 8 $IN $GT 2>&1 | grep -v amdgpu.ids | sed 's/^/C2  /' | tee gpurun_out/ab_gtab.log || exit 1
timeout -k 10 300 python tools/ab.py --rounds 8 --ndim 51 $IN $GT 2>&1 | grep -v amdgpu.ids | sed 's/^/51x51  /' | tee -a gpurun_out/ab_gtab.log || exit 1
bash tools/gpu_ab_c5.sh gtab "0 4" $IN $GT || exit 1
for v in "lds $IN" "gtab $GT"; do
  set -- $v
  echo "== $1" >> gpurun_out/strong_gtab.log
  RTHX_LIB=$2 bash tools/gpu_strong.sh >> gpurun_out/strong_gtab.log 2>&1 || { tail gpurun_out/strong_gtab.log; exit 1; }
done
cat gpurun_out/strong_gtab.log
