#!/bin/bash
# Diagnostic only: build ablated variants of the trace kernel (their results
# are WRONG) into csrc/_ablate/<mask>/librthx.so.  Time them with
#   RTHX_LIB=<path> python bench.py --no-cpu
# RTHX_ABLATE bits: 1 Philox 1 round, 2 no log, 4 no cospi, 8 no PIP test.
set -e
CSRC=$(cd $(dirname $0)/../raytraceheattransfer.jl_amd/csrc && pwd)
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden -munsafe-fp-atomics"
for m in "$@"; do
  d=$CSRC/_ablate/$m
  mkdir -p $d
  /opt/rocm/bin/hipcc $FLAGS -DRTHX_ABLATE=$m -c -o $d/k.o $CSRC/rthx_kernels.hip
  /opt/rocm/bin/hipcc $FLAGS -DRTHX_ABLATE=$m -x hip -c -o $d/a.o $CSRC/rthx_api.cpp
  g++ -O2 -std=c++17 -fPIC -ffp-contract=off -c -o $d/g.o $CSRC/rthx_grid.cpp
  /opt/rocm/bin/hipcc $FLAGS -shared -o $d/librthx.so $d/k.o $d/a.o $d/g.o
done
