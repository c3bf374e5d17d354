#!/bin/bash
# Variant of librthx.so with extra flags for the 3D view-factor kernel only.
#   bash tools/variant_vf.sh vf_fast -ffp-contract=fast -DRTHX_VF_WAVES=3
set -e
name=$1; shift
CSRC=$(cd $(dirname $0)/../raytraceheattransfer.jl_amd/csrc && pwd)
make -s -j8 -C $CSRC BUILD=_variants/$name VF3D_FLAGS="$*"
