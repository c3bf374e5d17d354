#!/bin/bash
# Large-N (hash tally) GPU tests, then the hash knob A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_large_n.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_large_n.log 2>&1 || { tail -40 gpurun_out/pytest_large_n.log; exit 1; }
tail -3 gpurun_out/pytest_large_n.log
bash tools/hash_ab.sh
