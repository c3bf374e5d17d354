"""Per-ray view of a trace kernel's SQ counters (tools/gpu_sq.sh output).

  python tools/sq_report.py sq.json RAYS [KERNEL_SUBSTRING]
"""
import json
import sys

d = json.load(open(sys.argv[1]))
rays = float(sys.argv[2])
name = sys.argv[3] if len(sys.argv) > 3 else "trace_exchange_kernel"
k = next(x for x in d if name in x)
c = {n: v["mean"] for n, v in d[k].items()}
wr = rays / 64.0  # wave-rays
print("kernel", k)
for n in sorted(c):
    print(f"  {n:26s} {c[n]:16.4g}   per wave-ray {c[n] / wr:10.2f}")
if "SQ_THREAD_CYCLES_VALU" in c and "SQ_ACTIVE_INST_VALU" in c:
    print("  lane utilisation (THREAD_CYCLES_VALU / (64*ACTIVE_INST_VALU)):",
          round(c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]), 3))
if "SQ_WAIT_ANY" in c and "SQ_WAVE_CYCLES" in c:
    print("  wait fraction:", round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 3),
          " issue-stall fraction:", round(c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"], 3))
