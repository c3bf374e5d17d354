#!/bin/bash
# GPU box: parity tests on the in-tree build, then an interleaved A/B of
# trace-kernel times (tools/ab.py) between the in-tree build and variants.
#   bash tools/ab_run.sh _variants/nopipe [more variant dirs...]
set -o pipefail
OUT=gpurun_out
CS=raytraceheattransfer.jl_amd/csrc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
libs="$CS/_build/librthx.so"
for v in "$@"; do libs="$libs $CS/$v/librthx.so"; done
timeout -k 10 300 python tools/ab.py --rounds 10 $libs 2>&1 | grep -v amdgpu.ids
