set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_c5.log 2>&1 || { tail -40 gpurun_out/pytest_c5.log; exit 1; }
tail -2 gpurun_out/pytest_c5.log
bash tools/c5_var_ab.sh main rf24 rf32 rf40
