"""Row-round quantisation of the C2 launch (diagnostic): trace-kernel time of
the first E emitter rows for several E around multiples of the resident
workgroup slots (256 CUs x 4 workgroups of 512 lanes = 1024 rows per round).

    python tools/tail_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import bench  # noqa: E402
from rthx import _lib, abi  # noqa: E402


def main():
    dom = bench.build_domain()
    flat = dom.flat()
    N = flat.n_emitters
    R = 100_000_000 // N
    dd = _lib.DeviceDomain(flat, 0)
    out = []
    for E in (1024, 2048, 4096, 8192, 9216, 9300, 9728, 10240, 10300, 10605):
        args, _keep = _lib.make_args(0, R, 10_000 * 2.220446049250313e-16, 1, 0, E, 1, device=0,
                                     flags=abi.RTHX_FLAG_DEVICE_ONLY)
        res = _lib.DeviceResult()
        for _ in range(20):
            res.trace(dd, args)
        ks = []
        for _ in range(40):
            res.trace(dd, args)
            ks.append(res.info()["trace_ms"])
        res.close()
        ks.sort()
        k = ks[len(ks) // 2]
        out.append({"rows": E, "kernel_ms": round(k, 4), "us_per_row": round(1e3 * k / E, 3)})
        print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
