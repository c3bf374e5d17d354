#!/bin/bash
# One GPU iteration (repo root, through gpurun): the GPU test suite, a bench
# line without the CPU leg, and (with SQ=1) the SQ counter passes of the
# trace kernel.  Every GPU step has its own time limit; the first failure
# ends the script.
#   bash tools/gpu_iter.sh TAG [pytest selection...]
set -o pipefail
TAG=${1:-iter}
shift
SEL=${*:-tests}
OUT=gpurun_out
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_$TAG.log 2>&1 || { tail -40 $OUT/pytest_$TAG.log; exit 1; }
tail -2 $OUT/pytest_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { tail -20 $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json
if [ "${SQ:-0}" = "1" ]; then
  bash tools/gpu_sq.sh $TAG || exit 1
fi
