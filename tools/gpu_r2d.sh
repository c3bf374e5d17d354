set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 tools/probe/valu_probe > gpurun_out/valu_probe_r2.json || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_boundary.py -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_boundary2.log 2>&1 || { tail -30 gpurun_out/pytest_boundary2.log; exit 1; }
tail -2 gpurun_out/pytest_boundary2.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_r2d.json 2> gpurun_out/bench_r2d.err || exit 1
cat gpurun_out/bench_r2d.json
timeout -k 10 200 python tools/bench_pipeline.py --repeat 3 > gpurun_out/pipeline_r2d.log 2>&1 || { cat gpurun_out/pipeline_r2d.log; exit 1; }
cat gpurun_out/pipeline_r2d.log
