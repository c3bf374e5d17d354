#!/bin/bash
# Direct-method variant: its GPU tests (RTHX_LIB=_ab/$1), then D1-D3 A/B against _build, alternating twice.
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out
C=raytraceheattransfer.jl_amd/csrc
RTHX_LIB=$C/_ab/$1/librthx.so timeout -k 10 400 python -u -m pytest tests/test_gpu_direct.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$1.log 2>&1 || { tail -30 gpurun_out/pytest_$1.log; exit 1; }
tail -n1 gpurun_out/pytest_$1.log
bash tools/gpu_r6_dab.sh _build "$@"
