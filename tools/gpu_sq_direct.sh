#!/bin/bash
# SQ counters of the direct-method kernel on one launch (2^24 rays) of a
# bench_direct.py case; per wave-leg summary.  Run on the GPU box from the repo root.
#   bash tools/gpu_sq_direct.sh D3
set -o pipefail
REPO=$(pwd)
OUT=$REPO/gpurun_out
CASE=${1:-D3}
TAG=direct_$CASE
RAYS=16777216
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_k_$TAG -o run -- python3 $REPO/tools/bench_direct.py --only $CASE --rays $RAYS --steps 3 --cpu-rays 0 > $OUT/prof_k_$TAG.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $OUT/prof_sqa_$TAG -o run -- python3 $REPO/tools/bench_direct.py --only $CASE --rays $RAYS --steps 1 --cpu-rays 0 > $OUT/prof_sqa_$TAG.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VMEM_WR --output-format csv -d $OUT/prof_sqb_$TAG -o run -- python3 $REPO/tools/bench_direct.py --only $CASE --rays $RAYS --steps 1 --cpu-rays 0 > $OUT/prof_sqb_$TAG.log 2>&1 || exit 1
cd $REPO
python tools/pmc_summary.py stats $OUT/prof_k_$TAG > $OUT/kstats_$TAG.json
python tools/pmc_summary.py pmc $OUT/prof_sqa_$TAG $OUT/prof_sqb_$TAG > $OUT/sq_$TAG.json
python tools/sq_report.py $OUT/sq_$TAG.json $RAYS trace_direct_kernel
