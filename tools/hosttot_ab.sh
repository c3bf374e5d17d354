set -o pipefail
V=$PWD/raytraceheattransfer.jl_amd/csrc/_variants/ep/librthx.so
for i in 1 2; do
  RTHX_LIB=$V timeout -k 10 120 python tools/step_overhead.py > gpurun_out/so_ep_$i.json || exit 1
  timeout -k 10 120 python tools/step_overhead.py > gpurun_out/so_main_$i.json || exit 1
  echo "ep $(cat gpurun_out/so_ep_$i.json)"; echo "main $(cat gpurun_out/so_main_$i.json)"
done
ONLY=C2,C3 STEPS=20 BINS=0 bash tools/cfg_ab.sh ep main ep main > gpurun_out/ht_ab.txt 2>&1 || exit 1
cat gpurun_out/ht_ab.txt
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_rel.log 2>&1; rc=$?; tail -3 gpurun_out/pt_rel.log; exit $rc
