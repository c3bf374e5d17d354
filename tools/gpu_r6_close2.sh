#!/bin/bash
# Round 6 closing, part 2, on the final tree: emulated strong shards
# (tools/gpu_strong.sh) and the C5 band pipeline over W = 8 emulated ranks
# with its rocprofv3 timeline (tools/gpu_r6_g.sh).
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_strong.sh > gpurun_out/strong_emulated_r6c.log 2>&1 || { tail gpurun_out/strong_emulated_r6c.log; exit 1; }
cat gpurun_out/strong_emulated_r6c.log
bash tools/gpu_r6_g.sh || exit 1
