#!/bin/bash
# Round SQ evidence (GPU box, repo root): VALU probe, SQ passes on the C2
# bench kernel, on one C5 band at 1e9 rays and on the 3D config-4 kernel.
#   bash tools/gpu_sq_round.sh TAG
set -o pipefail
TAG=${1:-r2}
bash tools/probe/run_probe.sh > /dev/null || exit 1
bash tools/gpu_sq.sh $TAG || exit 1
bash tools/gpu_sq_any.sh c5_$TAG trace_exchange_kernel 999956940 python3 $PWD/tools/bench_configs.py --only C5 --rays 1e9 --steps 1 --bins 0 --no-ramp || exit 1
bash tools/gpu_sq3d.sh sq3d_$TAG --ndim 10 --level 3 || exit 1
