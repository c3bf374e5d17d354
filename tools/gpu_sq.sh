#!/bin/bash
# SQ counter passes on the trace kernel (2 passes x 8 counters), then a per-ray summary.
set -o pipefail
REPO=$(pwd)
OUT=$REPO/gpurun_out
TAG=${1:-sq}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/prof_sqa_$TAG -o run -- python3 $REPO/bench.py --steps 2 --warmup 1 --no-cpu --faithful-steps 0 --philox10-steps 0 > $OUT/prof_sqa_$TAG.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 --output-format csv -d $OUT/prof_sqb_$TAG -o run -- python3 $REPO/bench.py --steps 2 --warmup 1 --no-cpu --faithful-steps 0 --philox10-steps 0 > $OUT/prof_sqb_$TAG.log 2>&1 || exit 1
cd $REPO
python tools/pmc_summary.py pmc $OUT/prof_sqa_$TAG $OUT/prof_sqb_$TAG > $OUT/sq_$TAG.json
python tools/sq_report.py $OUT/sq_$TAG.json 99994545
