#!/bin/bash
# Headline VALU trims (round 6): HEAD (f_surf wall lookup) against the
# working tree without (norot) and with (_build) the free-path word rotation;
# both carry the SGPR-held polynomial addends and the literal-scaled 1 - u.
# Parity tests of the headline path on the new build first.
export RTHX_DEV_KNOBS=1
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_numerics.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_valu.log 2>&1 || { tail -30 $OUT/pytest_valu.log; exit 1; }
tail -1 $OUT/pytest_valu.log
C=raytraceheattransfer.jl_amd/csrc
timeout -k 10 400 python tools/ab.py --rounds 20 $C/_ab/head/librthx.so $C/_ab/norot/librthx.so $C/_build/librthx.so 2>&1 | grep -v amdgpu.ids
