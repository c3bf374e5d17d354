"""Kernel time of C2 launches that hold only surface rows or only volume rows
(diagnostic): rows [0, 404) are the 404 wall elements, the rest the 10,201
cells.  Each launch of K rows (K below the resident workgroups) runs in one
round, so its time is one row's duration plus the launch's ramp.

  python tools/row_kind_cost.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytraceheattransfer.jl_amd"), os.path.join(ROOT, "tests"), ROOT]
import helpers as H  # noqa: E402
from rthx import _lib  # noqa: E402


def main():
    dom = H.square_domain(101)
    flat = dom.flat()
    N = flat.n_emitters
    R = 100_000_000 // N
    dd = _lib.DeviceDomain(flat, 0)
    res = _lib.DeviceResult()
    Ns = 404
    cases = [("surface rows 0-403", 0, Ns, 1), ("volume rows 404-807", Ns, 2 * Ns, 1),
             ("volume rows 5000-5403", 5000, 5000 + Ns, 1), ("all rows", 0, N, 1)]
    for name, b, e, s in cases:
        args, _k = _lib.make_args(0, R, H.NUDGE, 1, b, e, s, flags=_lib.abi.RTHX_FLAG_DEVICE_ONLY)
        for _ in range(3):
            res.trace(dd, args)
        ts = []
        for _ in range(10):
            res.trace(dd, args)
            ts.append(res.info()["trace_ms"])
        rows = (e - b + s - 1) // s
        print(f"{name:24s} rows {rows:6d}  kernel median {np.median(ts):.4f} ms  per row-slot {np.median(ts) / max(1, rows) * 1e3:.2f} us",
              flush=True)
    res.close()
    dd.close()


if __name__ == "__main__":
    main()
