"""Quick GPU probe used during development: parity on C1 and a timing of C2.

Usage: python tools/gpu_probe.py [rays_c2]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytraceheattransfer.jl_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle import oracle  # noqa: E402
from rthx import PolyVolume2D, RayTracingDomain2D, _lib  # noqa: E402

NUDGE = 10_000 * np.finfo(np.float64).eps


def square(nd, kappa=1.0, sigma=0.0):
    f = PolyVolume2D([(0.0, 0.0), (1.0, 0.0), (1.0, 1.0), (0.0, 1.0)], [True] * 4, 1, kappa, sigma)
    return RayTracingDomain2D([f], [(nd, nd)])


def run(dom, R, flags=0, seed=1):
    flat = dom.flat()
    args, keep = _lib.make_args(0, R, NUDGE, seed, 0, flat.n_emitters, flags=flags)
    dd = _lib.DeviceDomain(flat, 0)
    res = _lib.DeviceResult()
    res.trace(dd, args)
    out = res.csr() + (res.info(),)
    res.close()
    dd.close()
    return out, args, keep


def main():
    print("devices", _lib.device_count(), flush=True)
    for flags in (0, 1):
        dom = square(11)
        (rp, cols, cnt, info), args, keep = run(dom, 6060, flags)
        orp, ocols, ocnt, oinfo, _ = oracle.trace_exchange(dom.flat(), args, 16)
        same_rp = np.array_equal(rp, orp)
        same = same_rp and np.array_equal(cols, ocols) and np.array_equal(cnt, ocnt)
        print("C1 flags", flags, "identical:", same, "nnz", info["nnz"], oinfo["nnz"], "trace_ms", info["trace_ms"],
              "lost", info["lost_total"], oinfo["lost_total"], flush=True)
        if not same and same_rp:
            d = np.sum(cnt != ocnt)
            print("  count mismatches:", d, "abs diff sum", np.abs(cnt.astype(np.int64) - ocnt).sum())
    rays = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
    dom = square(101)
    N = dom.num_emitters
    R = rays // N
    flat = dom.flat()
    args, keep = _lib.make_args(0, R, NUDGE, 1, 0, N, flags=_lib.abi.RTHX_FLAG_DEVICE_ONLY)
    dd = _lib.DeviceDomain(flat, 0)
    res = _lib.DeviceResult()
    for it in range(4):
        t = time.time()
        res.trace(dd, args)
        info = res.info()
        wall = time.time() - t
        print(f"C2 it{it}: rays {info['rays_traced']} trace {info['trace_ms']:.2f} ms pack {info['pack_ms']:.2f} ms "
              f"wall {wall*1e3:.1f} ms -> {info['rays_traced']/info['trace_ms']/1e3:.1f} Mray/s (trace) "
              f"nnz {info['nnz']} lost {info['lost_total']}", flush=True)
    res.close()
    dd.close()


if __name__ == "__main__":
    main()
