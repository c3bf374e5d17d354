set -o pipefail
ONLY=C2,C3 STEPS=10 BINS=0 bash tools/cfg_ab.sh head main head main > gpurun_out/ek_ab.txt 2>&1 || exit 1
timeout -k 10 120 python tools/step_overhead.py > gpurun_out/step_overhead.json 2>gpurun_out/step_overhead.err || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_large_n.py > gpurun_out/ek_pytest.log 2>&1 || { tail -30 gpurun_out/ek_pytest.log; exit 1; }
tail -2 gpurun_out/ek_pytest.log
