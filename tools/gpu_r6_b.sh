#!/bin/bash
# Round 6: the row-sharded C5 band pipeline -- its GPU tests, the one-GPU
# emulation of W = 8 at 1e9 rays per band (every rank), and a rocprofv3
# kernel trace of the emulated rank that owns the last band.
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bands.py \
  > gpurun_out/r6/pytest_bands.log 2>&1 || { tail -30 gpurun_out/r6/pytest_bands.log; exit 1; }
tail -3 gpurun_out/r6/pytest_bands.log
timeout -k 10 600 python -u tools/bench_c5_bands.py --emulate-world 8 --pipeline --rays 1e9 \
  > gpurun_out/r6/c5_pipeline.log 2>&1 || { tail -30 gpurun_out/r6/c5_pipeline.log; exit 1; }
grep -v "^    " gpurun_out/r6/c5_pipeline.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_pipe -o run -- \
  python3 tools/bench_c5_bands.py --emulate-world 8 --pipeline --rays 1e9 --ranks 7 --reps 1 \
  > gpurun_out/r6/c5_pipeline_prof.log 2>&1 || { tail -30 gpurun_out/r6/c5_pipeline_prof.log; exit 1; }
find gpurun_out/r6/prof_pipe -name "*.csv" | head
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_accuracy.py \
  "tests/test_gpu_parity.py::test_philox10_build_exact" > gpurun_out/r6/pytest_acc.log 2>&1 || { tail -30 gpurun_out/r6/pytest_acc.log; exit 1; }
grep -E "RMS|C&S|passed|failed" gpurun_out/r6/pytest_acc.log
RTHX_ACCURACY_RECORD=gpurun_out/r6/accuracy.json timeout -k 10 600 python -u -m pytest -x -q -s --timeout 400 --timeout-method thread -m gpu \
  "tests/test_gpu_accuracy.py::test_f_smooth_rms_vs_1e9_ray_reference" > gpurun_out/r6/pytest_acc_rec.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu --steps 20 --warmup 10 > gpurun_out/r6/bench_a.json 2> gpurun_out/r6/bench_a.err || { tail gpurun_out/r6/bench_a.err; exit 1; }
python -c "
import json; d = json.load(open('gpurun_out/r6/bench_a.json'))
print('value', d['value'], 'kernel', d['roofline']['avg_kernel_ms'], 'philox10', d['philox10'])"
