#!/bin/bash
# GPU box: VALU issue-rate probe (plain run + one SQ counter pass to pin the
# counters' units against known instruction counts).
set -o pipefail
OUT=$(pwd)/gpurun_out
P=$(pwd)/tools/probe/valu_probe
export TMPDIR=/tmp
timeout -k 10 60 $P > $OUT/valu_probe.json || exit 1
cat $OUT/valu_probe.json
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_THREAD_CYCLES_VALU SQ_WAVES --output-format csv -d $OUT/prof_probe -o run -- $P > $OUT/prof_probe.log 2>&1 || exit 1
cd - > /dev/null
python tools/pmc_summary.py pmc $OUT/prof_probe > $OUT/sq_probe.json && cat $OUT/sq_probe.json
