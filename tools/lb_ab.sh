#!/bin/bash
# GPU box: 2D parity tests with the direct-CSR look-back, then the C2 bench
# with and without it (RTHX_NO_LOOKBACK=1), W = 1 and an emulated W = 2 shard.
set -o pipefail
OUT=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_accuracy.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/lb.log 2>&1 || { tail -30 $OUT/lb.log; exit 1; }
tail -1 $OUT/lb.log
for mode in 0 1; do
  for w in 1 2; do
    EW=""; [ $w -gt 1 ] && EW="--emulate-world $w"
    RTHX_NO_LOOKBACK=$mode timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu $EW 2>/dev/null > $OUT/lb.json || exit 1
    python3 -c "
import json; d=json.load(open('$OUT/lb.json')); v=d['value'] or d['rank0_mrays_s']
print('no_lookback=$mode W=$w %8.1f Grays/s per GPU  %.4f ms/step  trace %.4f ms  pack %.4f ms' % (v/1e3, d['ms_per_step'], d['roofline']['avg_kernel_ms'], d['pack_ms']))"
  done
done
