"""VALU issue floor of one kernel from its SQ counters, priced at the issue
rates of tools/probe/valu_probe.hip (profiles/round1/valu_probe.json).

  python tools/issue_floor.py sq.json RAYS_PER_LAUNCH KERNEL_SUBSTRING [kernel_ms]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
d = json.load(open(sys.argv[1]))
rays = float(sys.argv[2])
k = next(x for x in d if sys.argv[3] in x)
c = {n: v["mean"] for n, v in d[k].items()}
rates = json.load(open(os.path.join(ROOT, "profiles", "round1", "valu_probe.json")))["rates_wave_instr_per_s"]
f64 = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_FMA_F64"]
trans = c["SQ_INSTS_VALU_TRANS_F64"]
other = c["SQ_INSTS_VALU"] - f64 - trans
t = f64 / rates["v_fma_f64"] + trans / rates["v_rcp_f64"] + other / rates["v_fma_f32"]
wr = rays / 64.0
print(f"  VALU per wave-ray: fp64 {f64 / wr:.1f}, fp64 trans {trans / wr:.1f}, other {other / wr:.1f}")
print(f"  issue floor per launch: {t * 1e3:.3f} ms" + (f"  = {t * 1e3 / float(sys.argv[4]):.3f} of {sys.argv[4]} ms"
                                                     if len(sys.argv) > 4 else ""))
