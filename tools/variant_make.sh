#!/bin/bash
# Full librthx.so of git revision REV (or the working tree: REV=.) built by the
# csrc Makefile into csrc/_ab/<name>/ (git-ignored; it travels to the GPU box, so delete it after the A/B) (A/B timing with RTHX_LIB=...).
#   tools/variant_make.sh <name> <rev|.> [make VAR=value ...]
export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -e
name=$1; rev=$2; shift 2
ROOT=$(cd $(dirname $0)/.. && pwd)
d=$ROOT/raytraceheattransfer.jl_amd/csrc/_ab/$name
mkdir -p $d
if [ "$rev" = "." ]; then
  make -s -j8 -C $ROOT/raytraceheattransfer.jl_amd/csrc BUILD=$d "$@"
else
  tmp=$(mktemp -d)
  git -C $ROOT archive $rev raytraceheattransfer.jl_amd/csrc include | tar -x -C $tmp
  make -s -j8 -C $tmp/raytraceheattransfer.jl_amd/csrc BUILD=$d "$@"
  rm -rf $tmp
fi
rm -f $d/*.o
ls -la $d/librthx.so
