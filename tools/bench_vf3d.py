"""Throughput of the analytic 3D view factors (rthx_view_factors_3d) on one
MI355X beside the CPU restatement on a bounded row sample (diagnostic).

  python tools/bench_vf3d.py [--ndim 10,20] [--steps 3] [--cpu-max-pairs 6e6]

The unit cube with every face split into Ndim x Ndim sub-faces
(test/test_3d_viewfactors.jl geometry): n = 6 Ndim^2 polygons, n (n - 1)
ordered pairs, 16 edge pairs each.
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

import json  # noqa: E402

import helpers as H  # noqa: E402
from rthx import ViewFactorDomain3D  # noqa: E402
from rthx.domain3d import view_factors_3d  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ndim", default="10,20")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cpu-max-pairs", type=float, default=6e6)
    ap.add_argument("--cpu-threads", type=int, default=16)
    args = ap.parse_args()
    ref = json.load(open(os.path.join(H.GOLDEN, "reference_3d.json")))
    for nd in [int(x) for x in args.ndim.split(",")]:
        dom = ViewFactorDomain3D(ref["cube_points"], ref["cube_faces"], nd, [0.0] * 6, [-1.0] * 6, [1.0] * 6)
        xyz, nv = dom.polygon_arrays()
        n = len(nv)
        view_factors_3d(xyz, nv)  # warm-up
        ks, cs = [], []
        for _ in range(args.steps):
            t = time.perf_counter()
            F, _a, info = view_factors_3d(xyz, nv)
            cs.append(time.perf_counter() - t)
            ks.append(info["kernel_ms"])
        k = float(np.median(ks))
        c = float(np.median(cs)) * 1e3
        pairs = n * (n - 1)
        line = (f"cube Ndim={nd:3d} n={n:6d} pairs={pairs:.3e}  kernel {k:.2f} ms ({pairs / k / 1e3:.1f} Mpairs/s)  "
                f"call {c:.2f} ms  rowsum err {np.max(np.abs(F.sum(axis=1) - 1)):.2e}")
        if pairs <= args.cpu_max_pairs:
            from oracle import oracle

            t = time.perf_counter()
            F0, _ = oracle.view_factors_3d(xyz, nv, args.cpu_threads)
            dt = time.perf_counter() - t
            line += (f"  | CPU restatement {args.cpu_threads} thr: {dt * 1e3:.0f} ms ({pairs / dt / 1e6:.3f} Mpairs/s), "
                     f"max |dF| {np.max(np.abs(F - F0)):.1e}")
        print(line, flush=True)


if __name__ == "__main__":
    main()
