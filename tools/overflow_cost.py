"""Cost of a direct-CSR overflow re-trace (diagnostic).

The direct CSR of a single-polygon launch is sized from the previous launch
of the same shape (nnz + 1/8 + 64K entries) or, for a first launch, from a
guess; rows that outgrow it write nothing and the host traces the same
launch again at the exact size (rthx_result_info.lookback_fallbacks counts
it, together with look-back stalls).  This traces C2 (1e8 rays) on fresh
result objects with the default first guess and with a tiny one
(RTHX_CSR_CAP=65536, every row past it re-traced), and on a warm result.

    python tools/overflow_cost.py
"""
import json
import os

os.environ.setdefault("RTHX_DEV_KNOBS", "1")  # (RTHX_CSR_CAP is a knob: rthx_common.h)
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import bench  # noqa: E402
from rthx import _lib, abi  # noqa: E402


def one(dd, args, cap=None, warm=0):
    if cap is not None:
        os.environ["RTHX_CSR_CAP"] = str(cap)
    else:
        os.environ.pop("RTHX_CSR_CAP", None)
    res = _lib.DeviceResult()
    try:
        for _ in range(warm):
            res.trace(dd, args)
        res.trace(dd, args)
        inf = res.info()
        return {"trace_ms": round(inf["trace_ms"], 4), "total_ms": round(inf["total_ms"], 4),
                "lookback_fallbacks": inf["lookback_fallbacks"], "nnz": inf["nnz"]}
    finally:
        res.close()


def main():
    dom = bench.build_domain()
    flat = dom.flat()
    N = flat.n_emitters
    R = 100_000_000 // N
    dd = _lib.DeviceDomain(flat, 0)
    args, _keep = _lib.make_args(0, R, 10_000 * 2.220446049250313e-16, 1, 0, N, 1, device=0,
                                 flags=abi.RTHX_FLAG_DEVICE_ONLY)
    one(dd, args, warm=3)  # (module load, first-touch allocations)
    out = {"fresh_default_guess": one(dd, args), "fresh_tiny_guess_retrace": one(dd, args, cap=65536),
           "warm_sized_from_previous": one(dd, args, warm=2)}
    os.environ.pop("RTHX_CSR_CAP", None)
    dd.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
