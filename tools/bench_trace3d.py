"""Throughput of the 3D Monte Carlo tracer on BASELINE config 4 (cube +
icosphere surface enclosure, 1e8 rays, one MI355X) beside the CPU
restatement on a bounded row sample (diagnostic; bench.py's headline is the
2D tracer).

  python tools/bench_trace3d.py [--rays 1e8] [--ndim 10] [--level 3] [--steps 5]
  python tools/bench_trace3d.py --interior --level 3   # config 4's other enclosure:
      the inside of the readme's icosphere (readme.md:532-704), no cube
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
from rthx.trace3d import Scene3D  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=float, default=1e8)
    ap.add_argument("--ndim", type=int, default=10)
    ap.add_argument("--level", type=int, default=3)
    ap.add_argument("--radius", type=float, default=0.3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--cpu-rows", type=int, default=8)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-groups", action="store_true", help="every polygon its own group (no coplanar faces)")
    ap.add_argument("--interior", action="store_true", help="the inside of the readme's unit icosphere alone")
    args = ap.parse_args()
    if args.interior:  # rays leave the triangles toward the centre; every triangle sees every other
        pts, faces = H.icosphere_mesh(args.level)
        xyz = np.zeros((len(faces), 4, 3))
        for i, f in enumerate(faces):
            xyz[i, :3] = pts[f - 1]
            xyz[i, 3] = pts[f[2] - 1]
        nv = np.full(len(faces), 3, dtype=np.int32)
        nrm = -xyz[:, :3].mean(axis=1)
        nc = 0
        args.no_groups = True
    else:
        xyz, nv, nrm, nc = H.cube_icosphere_scene(args.ndim, args.level, args.radius)
    n = len(nv)
    R = int(args.rays) // n
    from rthx import _lib
    _lib.load().rthx_device_synchronize(0)  # HIP context up before the build is timed
    t = time.perf_counter()
    groups = None if args.no_groups else H.cube_icosphere_groups(args.ndim, args.level)
    t_groups = time.perf_counter() - t
    t = time.perf_counter()
    scene = Scene3D(xyz, nv, nrm, groups=groups)
    t_build = time.perf_counter() - t
    scene.trace(R, device_only=True)
    ks, cs = [], []
    for _ in range(args.steps):
        t = time.perf_counter()
        _, _, _, info = scene.trace(R, device_only=True)
        cs.append(time.perf_counter() - t)
        ks.append(info["trace_ms"])
    try:
        stats = scene.stats()
    except AttributeError:  # a variant library without rthx_scene3d_stats
        stats = {}
    k = float(np.median(ks))
    c = float(np.median(cs)) * 1e3
    rays = n * R
    what = (f"config4 icosphere interior L{args.level}" if args.interior else
            f"config4 cube {args.ndim}x{args.ndim}/face + icosphere L{args.level}")
    line = (f"{what} (n={n}, {n - nc} triangles, "
            f"{int(np.sum(np.where(nv == 4, 2, 1)))} MT triangles, {'polygon' if args.no_groups else 'face'} groups)  R={R} rays={rays:.3e}  scene build {t_build * 1e3:.0f} ms (groups {t_groups * 1e3:.0f} ms)  "
            f"BVH {stats}  kernel {k:.2f} ms ({rays / k / 1e6:.2f} Grays/s)  call {c:.2f} ms  lost {info['lost_total']}  nnz {info['nnz']}")
    if args.cpu_rows > 0:
        from oracle import oracle

        rows = args.cpu_rows
        stride = max(1, n // rows)
        Rc = 20_000
        t = time.perf_counter()
        oracle.trace_exchange_3d(xyz, nv, nrm, Rc, begin=0, end=rows * stride, stride=stride,
                                 nthreads=args.cpu_threads, groups=groups)
        dt = time.perf_counter() - t
        line += f"  | CPU restatement (brute force) {args.cpu_threads} thr: {rows * Rc / dt / 1e6:.3f} Mrays/s"
    print(line, flush=True)
    scene.close()


if __name__ == "__main__":
    main()
