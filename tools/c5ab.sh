set -o pipefail
OUT=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -2 $OUT/parity.log
for r in 1e8 1e9; do
  RTHX_LIB=raytraceheattransfer.jl_amd/csrc/_variants/base/librthx.so timeout -k 10 200 python tools/bench_configs.py --only C5 --steps 4 --rays $r 2>&1 | grep C5 | sed 's/^/base /'
  timeout -k 10 200 python tools/bench_configs.py --only C5 --steps 4 --rays $r 2>&1 | grep C5 | sed 's/^/clds /'
done
