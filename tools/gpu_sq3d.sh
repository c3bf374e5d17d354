#!/bin/bash
# SQ counter passes on the 3D tracer kernel (config 4, 1e8 rays), per-ray summary.
#   bash tools/gpu_sq3d.sh [tag] [extra bench_trace3d args]
set -o pipefail
REPO=$(pwd)
OUT=$REPO/gpurun_out
TAG=${1:-sq3d}
shift
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
B="python3 $REPO/tools/bench_trace3d.py --steps 1 --cpu-rows 0 $*"
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/prof_sqa_$TAG -o run -- $B > $OUT/prof_sqa_$TAG.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 --output-format csv -d $OUT/prof_sqb_$TAG -o run -- $B > $OUT/prof_sqb_$TAG.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_BUSY_CYCLES --output-format csv -d $OUT/prof_sqc_$TAG -o run -- $B > $OUT/prof_sqc_$TAG.log 2>&1 || exit 1
cd $REPO
python tools/pmc_summary.py pmc $OUT/prof_sqa_$TAG $OUT/prof_sqb_$TAG $OUT/prof_sqc_$TAG > $OUT/sq_$TAG.json
python tools/sq_report.py $OUT/sq_$TAG.json 1e8 trace_exchange_3d
