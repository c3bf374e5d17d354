"""C5 kernel time against rays per emitter and band (per-row overhead vs walk).

  python tools/c5_diag.py [--rs 1,100,2426,24268] [--bins 0,7]
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytraceheattransfer.jl_amd"), os.path.join(ROOT, "tests"), ROOT]
import helpers as H  # noqa: E402
from rthx import _lib, abi  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rs", default="1,100,2426,24268")
ap.add_argument("--bins", default="0,3,7")
ap.add_argument("--steps", type=int, default=3)
args = ap.parse_args()
dom = H.greenhouse_domain()
flat = dom.flat()
N = flat.n_emitters
dd = _lib.DeviceDomain(flat, 0)
res = _lib.DeviceResult()
for b in (int(x) for x in args.bins.split(",")):
    for R in (int(x) for x in args.rs.split(",")):
        a, _k = _lib.make_args(b, R, H.NUDGE, 1, 0, N, 1, flags=abi.RTHX_FLAG_DEVICE_ONLY)
        res.trace(dd, a)
        t = []
        for _ in range(args.steps):
            res.trace(dd, a)
            t.append(res.info()["trace_ms"])
        k = float(np.median(t))
        print(f"band {b} R {R:6d} kernel {k:8.3f} ms  {N * R / k / 1e6:8.2f} Grays/s  us/row*CU {k * 1e3 * 256 / N:7.2f}",
              flush=True)
res.close()
dd.close()
