#!/bin/bash
# Round 6: the row-sharded C5 band pipeline -- its GPU tests, the one-GPU
# emulation of W = 8 at 1e9 rays per band (every rank; the last band whole
# and in 2 pieces), a rocprofv3 kernel trace of the emulated rank that owns
# the last band; the Philox-10 build's parity, the faithful accuracy bar and
# a bench line.
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bands.py \
  "tests/test_gpu_parity.py::test_philox10_build_exact" > gpurun_out/r6/pytest_bands.log 2>&1 || { tail -30 gpurun_out/r6/pytest_bands.log; exit 1; }
tail -3 gpurun_out/r6/pytest_bands.log
for P in 1 2; do
  timeout -k 10 600 python -u tools/bench_c5_bands.py --emulate-world 8 --pipeline --rays 1e9 --last-parts $P \
    > gpurun_out/r6/c5_pipeline_P$P.log 2>&1 || { tail -30 gpurun_out/r6/c5_pipeline_P$P.log; exit 1; }
  grep -v "^    " gpurun_out/r6/c5_pipeline_P$P.log | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_pipe -o run --output-format csv -- \
  python3 tools/bench_c5_bands.py --emulate-world 8 --pipeline --rays 1e9 --ranks 7 --reps 1 --last-parts 2 \
  > gpurun_out/r6/c5_pipeline_prof.log 2>&1 || { tail -30 gpurun_out/r6/c5_pipeline_prof.log; exit 1; }
find gpurun_out/r6/prof_pipe -name "*.csv" | head
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_accuracy.py \
  > gpurun_out/r6/pytest_acc.log 2>&1 || { tail -30 gpurun_out/r6/pytest_acc.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6/pytest_acc.log | tail -2
RTHX_ACCURACY_RECORD=gpurun_out/r6/accuracy.json timeout -k 10 600 python -u -m pytest -x -q -s --timeout 400 --timeout-method thread -m gpu \
  "tests/test_gpu_accuracy.py::test_f_smooth_rms_vs_1e9_ray_reference" > gpurun_out/r6/pytest_acc_rec.log 2>&1 || exit 1
grep RMS gpurun_out/r6/pytest_acc_rec.log
timeout -k 10 400 python bench.py > gpurun_out/r6/bench_a.json 2> gpurun_out/r6/bench_a.err || { tail gpurun_out/r6/bench_a.err; exit 1; }
python -c "
import json; d = json.load(open('gpurun_out/r6/bench_a.json'))
print('value', d['value'], 'kernel', d['roofline']['avg_kernel_ms'], 'philox10', d['philox10'], 'faithful', d['faithful_sampling']['value'])"
