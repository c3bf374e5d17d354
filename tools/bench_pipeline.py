"""The whole device pipeline on a BASELINE config (diagnostic): mesh(N;
method=:exchange) = trace + F_raw (normalised on the device) to the host +
smooth_F of the device-resident counts, then solveEquilibrium! (grey GERT
solve) on the device-resident F_smooth; last, the host copy of F_smooth.

  python tools/bench_pipeline.py [--ndim 101] [--rays 1e8]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytraceheattransfer.jl_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import helpers as H  # noqa: E402
from rthx.equilibrium import solve_equilibrium  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ndim", type=int, default=101)
    ap.add_argument("--rays", type=float, default=1e8)
    ap.add_argument("--repeat", type=int, default=2)
    a = ap.parse_args()
    for r in range(a.repeat):
        dom = H.square_domain(a.ndim)
        t0 = time.perf_counter()
        dom(int(a.rays), seed=1 + r, verbose=False)
        t_first = time.perf_counter() - t0
        # steady state: mesh() again on the same domain (flattened descriptor
        # and device upload cached, as the reference builds its grids once)
        t0 = time.perf_counter()
        dom(int(a.rays), seed=1 + r, verbose=False)
        t1 = time.perf_counter()
        info = {}
        from rthx.equilibrium import equilibrium_grey
        T, j, Abs, rr = equilibrium_grey(dom, None, info=info)  # F_smooth read in place on the device
        t2 = time.perf_counter()
        _ = dom.F_smooth  # host copy on first access
        t3 = time.perf_counter()
        _ = dom.F_raw  # host copy on first access
        t4 = time.perf_counter()
        sm = getattr(dom, "last_smooth_info", {})
        tr = dom.last_trace_info[0]
        print(f"ndim {a.ndim} rays {a.rays:.0e}: mesh() {1e3 * (t1 - t0):.0f} ms (first call on a new domain "
              f"{1e3 * t_first:.0f} ms: flattening + upload; trace kernel "
              f"{tr['trace_ms']:.2f} ms), solve {1e3 * (t2 - t1):.0f} ms (GMRES {info['iterations']} iterations, "
              f"library {info['ms_total']:.1f} ms, residual {info['residual']:.2e}), energy error "
              f"{dom.energy_error:.2e}; smoothing library {sm.get('ms_total', float('nan')):.1f} ms (OP "
              f"{sm.get('ms_op', float('nan')):.1f}, AP {sm.get('ms_ap', float('nan')):.1f}, {sm.get('ap_iters')} "
              f"iterations); on first read: F_smooth to the host {1e3 * (t3 - t2):.0f} ms, F_raw "
              f"{1e3 * (t4 - t3):.0f} ms", flush=True)


if __name__ == "__main__":
    main()
