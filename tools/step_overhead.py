"""Host overhead of one bench step (the blocking rthx_trace_exchange call) on
the headline workload: wall time per call vs the trace kernel's HIP-event
time, with and without the per-step rthx_result_get_info in the loop.

    python tools/step_overhead.py [--calls 200]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import bench  # noqa: E402
from rthx import _lib, abi  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--rays", type=float, default=1e8)
    a = ap.parse_args()
    dom = bench.build_domain()
    flat = dom.flat()
    N = flat.n_emitters
    R = int(a.rays) // N
    dd = _lib.DeviceDomain(flat, 0)
    args, _keep = _lib.make_args(0, R, 10_000 * 2.220446049250313e-16, 1, 0, N, 1, device=0, flags=abi.RTHX_FLAG_DEVICE_ONLY)
    res = _lib.DeviceResult()
    for _ in range(50):
        res.trace(dd, args)
    out = {}
    for mode in ("trace", "trace+info", "trace", "trace+info"):
        _lib.synchronize(0)
        ks = []
        t0 = time.perf_counter()
        for _ in range(a.calls):
            res.trace(dd, args)
            if mode == "trace+info":
                ks.append(res.info()["trace_ms"])
        wall = (time.perf_counter() - t0) / a.calls * 1e3
        if not ks:
            ks = [res.info()["trace_ms"]]
        k = sum(ks) / len(ks)
        out.setdefault(mode, []).append({"wall_ms": round(wall, 4), "kernel_ms": round(k, 4),
                                         "gap_ms": round(wall - k, 4)})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
