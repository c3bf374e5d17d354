#!/bin/bash
# Build csrc/ as of git revision REV into csrc/_variants/<name>/librthx.so.
set -e
name=$1; rev=$2; shift 2
ROOT=$(cd $(dirname $0)/.. && pwd)
tmp=$(mktemp -d)
git -C $ROOT archive $rev raytraceheattransfer.jl_amd/csrc include | tar -x -C $tmp
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fvisibility=hidden -munsafe-fp-atomics"
C=$tmp/raytraceheattransfer.jl_amd/csrc
d=$ROOT/raytraceheattransfer.jl_amd/csrc/_variants/$name
mkdir -p $d
/opt/rocm/bin/hipcc $FLAGS -ffp-contract=fast $* -c -o $d/k.o $C/rthx_kernels.hip
/opt/rocm/bin/hipcc $FLAGS -x hip -c -o $d/a.o $C/rthx_api.cpp
g++ -O2 -std=c++17 -fPIC -ffp-contract=off -c -o $d/g.o $C/rthx_grid.cpp
/opt/rocm/bin/hipcc $FLAGS -shared -o $d/librthx.so $d/k.o $d/a.o $d/g.o
rm -rf $tmp
