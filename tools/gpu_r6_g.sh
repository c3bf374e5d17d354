#!/bin/bash
# Round 6: the C5 band pipeline with the assembly order (most transparent
# band last) and device copy-outs on the library's copy stream: GPU tests,
# the W = 8 emulation (last band whole / in 2 pieces), a rocprofv3 kernel
# trace of the emulated rank that owns the last band.
export RTHX_DEV_KNOBS=1
set -o pipefail
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bands.py \
  tests/test_gpu_boundary.py > gpurun_out/r6/pytest_bands_g.log 2>&1 || { tail -30 gpurun_out/r6/pytest_bands_g.log; exit 1; }
tail -2 gpurun_out/r6/pytest_bands_g.log
for P in 1 2; do
  timeout -k 10 600 python -u tools/bench_c5_bands.py --emulate-world 8 --pipeline --rays 1e9 --last-parts $P \
    > gpurun_out/r6/c5_pipeline_g_P$P.log 2>&1 || { tail -30 gpurun_out/r6/c5_pipeline_g_P$P.log; exit 1; }
  grep -v "^    " gpurun_out/r6/c5_pipeline_g_P$P.log | cut -c1-220
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/r6/prof_pipe_g
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r6/prof_pipe_g -o run --output-format csv -- \
  python3 tools/bench_c5_bands.py --emulate-world 8 --pipeline --rays 1e9 --ranks 7 --reps 1 --last-parts 2 \
  > gpurun_out/r6/c5_pipeline_g_prof.log 2>&1 || { tail -30 gpurun_out/r6/c5_pipeline_g_prof.log; exit 1; }
python tools/pipeline_timeline.py gpurun_out/r6/prof_pipe_g/run_kernel_trace.csv --skip 14 --traces 9 | tail -4
