#!/bin/bash
# Build the current csrc/ into csrc/_variants/<name>/librthx.so (for A/B timing
# on the GPU with RTHX_LIB=...).  Extra args are passed as compiler flags.
set -e
name=$1; shift
CSRC=$(cd $(dirname $0)/../raytraceheattransfer.jl_amd/csrc && pwd)
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden -munsafe-fp-atomics"
KFLAGS="-ffp-contract=fast $*"
d=$CSRC/_variants/$name
mkdir -p $d
/opt/rocm/bin/hipcc $FLAGS $KFLAGS -c -o $d/k.o $CSRC/rthx_kernels.hip
/opt/rocm/bin/hipcc $FLAGS -x hip -c -o $d/a.o $CSRC/rthx_api.cpp
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -c -o $d/g.o $CSRC/rthx_grid.cpp
/opt/rocm/bin/hipcc $FLAGS -shared -o $d/librthx.so $d/k.o $d/a.o $d/g.o
