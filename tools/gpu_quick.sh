#!/bin/bash
# quick GPU iteration: parity tests then a bench line (no CPU leg)
set -o pipefail
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?
tail -5 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" $OUT/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu ${BENCH_ARGS} > $OUT/bench_quick.json 2> $OUT/bench_quick.err
rc=$?
cat $OUT/bench_quick.json; tail -3 $OUT/bench_quick.err
exit $rc
