"""Throughput of method=:direct (rthx_trace_direct) on one MI355X, beside the
CPU restatement on a bounded sample (diagnostic; the headline line is bench.py).

  python tools/bench_direct.py [--rays 1e8] [--steps 5] [--cpu-rays 2e6]

D1  C&S 101x101 grey, kappa=1, black walls, re-emitting gas      (C2's domain)
D2  51x51 kappa=1 sigma_s=5, walls epsilon=0.5                   (C3's domain, multi-bounce)
D3  C&S 11x11 grey (the reference's test size)
Reports rays/s and legs/s (one leg = one traceRay call: 1 + path events).
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
from rthx import _lib  # noqa: E402
from rthx import direct as DR  # noqa: E402

CASES = {
    "D1": lambda: H.square_domain(101),
    "D2": lambda: H.square_domain(51, kappa=1.0, sigma_s=5.0, epsilon=0.5),
    "D3": lambda: H.square_domain(11),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=float, default=1e8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-rays", type=float, default=2e6)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--only", default="D1,D2,D3")
    args = ap.parse_args()
    rays = int(args.rays)
    for name in args.only.split(","):
        dom = CASES[name]()
        w, _ = DR.prepare_emitters(dom)
        eps, om, re = DR.element_data(dom)
        dd = _lib.device_domain(dom, 0)
        a = DR.make_direct_args(0, rays, H.NUDGE, 1)
        DR.trace_direct_counts(dd, w, eps, om, re, a)  # warm-up (same launches as the timed calls)
        ks, cs = [], []
        for _ in range(args.steps):
            t = time.perf_counter()
            _c, info = DR.trace_direct_counts(dd, w, eps, om, re, a)
            cs.append(time.perf_counter() - t)
            ks.append(info["trace_ms"])
        k = float(np.median(ks))
        c = float(np.median(cs)) * 1e3
        legs = rays + info["events"]
        line = (f"{name} n={dom.num_emitters:6d} rays={rays:.2e} events/ray={info['events'] / rays:.2f}  "
                f"kernel {k:.2f} ms ({rays / k / 1e6:.2f} Grays/s, {legs / k / 1e6:.2f} Glegs/s)  "
                f"call {c:.2f} ms  replayed {info['replayed']}")
        if args.cpu_rays > 0:
            from oracle import oracle

            cr = int(args.cpu_rays)
            t = time.perf_counter()
            oracle.trace_direct(dom.flat(), w, eps, om, re, DR.make_direct_args(0, cr, H.NUDGE, 1), args.cpu_threads)
            dt = time.perf_counter() - t
            line += f"  | CPU oracle {args.cpu_threads} thr: {cr / dt / 1e6:.2f} Mrays/s ({cr:.0e} rays)"
        print(line, flush=True)


if __name__ == "__main__":
    main()
