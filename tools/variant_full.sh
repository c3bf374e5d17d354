#!/bin/bash
# Build the whole librthx.so from the current csrc/ into
# csrc/_variants/<name>/librthx.so with extra trace-kernel flags (A/B timing
# with RTHX_LIB=... in separate processes).
#   bash tools/variant_full.sh refill32 -DRTHX_DIRECT_REFILL=32
set -e
name=$1; shift
CSRC=$(cd $(dirname $0)/../raytraceheattransfer.jl_amd/csrc && pwd)
make -s -j8 -C $CSRC BUILD=_variants/$name KERNEL_FLAGS="-ffp-contract=fast $*"
