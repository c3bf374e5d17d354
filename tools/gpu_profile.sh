#!/bin/bash
# Round profiling recipe (run on the GPU box through gpurun from the repo root):
#   bench line, rocprofv3 kernel-trace stats, and separate --pmc passes.
set -e -o pipefail
REPO=$(pwd)
OUT=$REPO/gpurun_out
TAG=${1:-r1}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 420 python $REPO/bench.py --steps 20 --warmup 3 > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_stats_$TAG -o run -- python3 $REPO/bench.py --steps 10 --warmup 2 --no-cpu --faithful-steps 0 --philox10-steps 0 > $OUT/prof_stats_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/prof_fetch_$TAG -o run -- python3 $REPO/bench.py --steps 3 --warmup 1 --no-cpu --faithful-steps 0 --philox10-steps 0 > $OUT/prof_fetch_$TAG.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/prof_write_$TAG -o run -- python3 $REPO/bench.py --steps 3 --warmup 1 --no-cpu --faithful-steps 0 --philox10-steps 0 > $OUT/prof_write_$TAG.log 2>&1

cd $REPO
python tools/pmc_summary.py stats $OUT/prof_stats_$TAG > $OUT/stats_$TAG.json
python tools/pmc_summary.py traffic $OUT/prof_fetch_$TAG $OUT/prof_write_$TAG $OUT/traffic_$TAG.json > /dev/null

cat $OUT/bench_$TAG.json
