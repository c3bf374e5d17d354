"""Throughput of the trace on every BASELINE.json GPU config (diagnostic; the
headline line is bench.py).  One MI355X, inputs resident, CSR left on the
device; median trace-kernel time (HIP events) and whole-call time.

  python tools/bench_configs.py [--rays 1e8] [--steps 10]

C2  101x101 grey kappa=1                       (bench.py's workload)
C3  51x51 kappa=1 sigma_s=5 (beta=6)            exchange path: no re-scatter
C5  201x201 8-band greenhouse, 67 layers        every band spatially non-uniform;
                                               rays per band as the reference
                                               (parallelRayTracing.jl:6,22)
L301 301x301 grey kappa=1 (N = 91805)          large N: LDS hash row tallies
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytraceheattransfer.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import helpers as H  # noqa: E402
from rthx import _lib, abi  # noqa: E402


def run(name, dom, rays, steps, bins=(0,)):
    """Median kernel and call time per band; with several bands (C5) every
    band's line and the whole configuration: all bands' rays over the sum of
    the bands' median times (a mean or median band would hide the slow
    bands)."""
    flat = dom.flat()
    N = flat.n_emitters
    R = rays // N
    dd = _lib.DeviceDomain(flat, 0)
    res = _lib.DeviceResult()
    tot_k = tot_c = 0.0
    for b in bins:
        a, _k = _lib.make_args(b, R, H.NUDGE, 1, 0, N, 1, flags=abi.RTHX_FLAG_DEVICE_ONLY)
        for _ in range(3):
            res.trace(dd, a)
        t_k, t_c = [], []
        for _ in range(steps):
            t = time.perf_counter()
            res.trace(dd, a)
            t_c.append(time.perf_counter() - t)
            t_k.append(res.info()["trace_ms"])
        k = float(np.median(t_k))
        c = float(np.median(t_c)) * 1e3
        tot_k += k
        tot_c += c
        info = res.info()
        tag = f"{name} band {b}" if len(bins) > 1 else name
        print(f"{tag:10s} N={N:6d} R={R:6d} rays={N * R:.3e}  kernel {k:.3f} ms ({N * R / k / 1e6:.1f} Grays/s)  "
              f"call {c:.3f} ms ({N * R / c / 1e6:.1f} Grays/s)  nnz {info['nnz']}", flush=True)
    if len(bins) > 1:
        rays_all = len(bins) * N * R
        print(f"{name} total: {len(bins)} bands, {rays_all:.3e} rays  kernels {tot_k:.1f} ms "
              f"({rays_all / tot_k / 1e6:.2f} Grays/s)  calls {tot_c:.1f} ms ({rays_all / tot_c / 1e6:.2f} Grays/s)",
              flush=True)
    res.close()
    dd.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=float, default=1e8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--only", default="C2,C3,C5")
    ap.add_argument("--bins", default="0,1,2,3,4,5,6,7", help="C5 bands (0-based)")
    ap.add_argument("--no-ramp", action="store_true", help="skip the C2 clock ramp (counter passes)")
    args = ap.parse_args()
    only = args.only.split(",")
    rays = int(args.rays)
    # GPU clock ramp: trace the C2 row set for 0.3 s before timing anything
    dom = H.square_domain(101)
    flat = dom.flat()
    dd = _lib.DeviceDomain(flat, 0)
    res = _lib.DeviceResult()
    a, _k = _lib.make_args(0, 9429, H.NUDGE, 1, 0, flat.n_emitters, 1, flags=abi.RTHX_FLAG_DEVICE_ONLY)
    t = time.perf_counter()
    while not args.no_ramp and time.perf_counter() - t < 0.3:
        res.trace(dd, a)
    res.close()
    dd.close()
    if "C2" in only:
        run("C2", H.square_domain(101), rays, args.steps)
    if "C3" in only:
        run("C3", H.square_domain(51, kappa=1.0, sigma_s=5.0), rays, args.steps)
    if "L301" in only:
        run("L301", H.square_domain(301), rays, args.steps)
    if "C5" in only:
        run("C5", H.greenhouse_domain(), rays, max(1, args.steps // 4), bins=tuple(int(b) for b in args.bins.split(",")))


if __name__ == "__main__":
    main()
