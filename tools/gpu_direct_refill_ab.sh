export RTHX_DEV_KNOBS=1  # (librthx honours RTHX_* knobs only with this set: rthx_common.h knob)
set -o pipefail
A=raytraceheattransfer.jl_amd/csrc
for r in 1 2; do
for L in _build/librthx.so _ab/dr8/librthx.so _ab/dr24/librthx.so _ab/dr32/librthx.so; do
  RTHX_LIB=$A/$L timeout -k 10 120 python tools/bench_direct.py --only D1,D2 --cpu-rays 0 --steps 5 2>&1 | grep -v amdgpu | sed "s|^|$L |" || exit 1
done; done
