#!/bin/bash
# Closing evidence of round 2: smoke, full GPU suite + bench + rocprof + PMC +
# configs + 3D (round_refresh), large-N and C5 band tables, SQ of the headline.
set -o pipefail
OUT=gpurun_out
TAG=${1:-r2d}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
grep smoke $OUT/smoke.log
bash tools/round_refresh.sh $TAG || exit 1
timeout -k 10 200 python tools/bench_configs.py --only L301 >> $OUT/configs.log 2>&1 || exit 1
timeout -k 10 200 python tools/bench_configs.py --only L301 --rays 9e8 --steps 3 >> $OUT/configs.log 2>&1 || exit 1
grep L301 $OUT/configs.log
timeout -k 10 300 python tools/bench_c5_bands.py > $OUT/c5_bands.log 2>&1 || exit 1
grep -v amdgpu $OUT/c5_bands.log
bash tools/gpu_sq.sh $TAG > $OUT/sq_$TAG.log 2>&1 || exit 1
grep "VALU \|lane\|wait" $OUT/sq_$TAG.log
