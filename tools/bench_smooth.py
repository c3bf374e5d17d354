"""Smoothing throughput (smooth_F on the device) on the C2 workload
(diagnostic): trace 1e8 rays on the GPU, then time rthx_smooth_F on F_raw.

  python tools/bench_smooth.py [--ndim 101] [--rays 1e8] [--repeat 3]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytraceheattransfer.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import helpers as H  # noqa: E402
from rthx.exchange import exchange_ray_tracing  # noqa: E402
from rthx.smoothing import get_w, smooth_F  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ndim", type=int, default=101)
    ap.add_argument("--rays", type=float, default=1e8)
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--k-dykstra", type=int, default=None)
    a = ap.parse_args()
    dom = H.square_domain(a.ndim)
    t = time.perf_counter()
    F = exchange_ray_tracing(dom, int(a.rays), H.NUDGE, False, None, seed=1)
    print(f"trace + CSR to host: {time.perf_counter() - t:.3f} s, N={F.shape[0]} nnz={F.nnz} "
          f"density={F.nnz / F.shape[0] ** 2:.3f}", flush=True)
    w = get_w(dom)
    for r in range(a.repeat):
        info = {}
        t = time.perf_counter()
        Fs = smooth_F(F, w, dom.num_surfaces, verbose=(r == 0), info=info, k_dykstra=a.k_dykstra)
        dt = time.perf_counter() - t
        n = info["n"]
        # dense AP reads and writes the upper triangle once per iteration (k_ap_sym)
        ap_bytes = info["ap_iters"] * 16.0 * n * (n + 1) / 2
        print(f"smooth_F: {dt * 1e3:.1f} ms wall (library {info['ms_total']:.1f} ms: OP {info['ms_op']:.1f}, "
              f"AP {info['ms_ap']:.1f} ms, {info['ap_iters']} AP iterations, {info['pcg_iters']} PCG), "
              f"AP scale+sum traffic {ap_bytes / info['ms_ap'] / 1e6:.0f} GB/s lower bound, "
              f"dense={info['dense']} chi={info['chi']:.3f} converged={info['converged']}", flush=True)
    Fd = Fs if isinstance(Fs, np.ndarray) else Fs.toarray()
    print("row-sum error", float(np.abs(Fd.sum(axis=1) - 1).max()), "min", float(Fd.min()))


if __name__ == "__main__":
    main()
