"""C5 (BASELINE configs[4]) with its bands over the visible GPUs: mesh()'s
trace half (smooth=False) of the 201x201 8-band greenhouse at R rays per band,
band per GPU (rthx.exchange band workers, one host thread per device).

  python tools/bench_c5_bands.py [--rays 1e9] [--devices 0,1,...]  (default: every visible device)

Prints the whole-call rate (all bands, all devices) and each band's kernel time.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "raytraceheattransfer.jl_amd"), os.path.join(ROOT, "tests"), ROOT]
import helpers as H  # noqa: E402
from rthx import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rays", type=float, default=1e9)
    ap.add_argument("--devices", default="")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--rows", action="store_true", help="split each band's rows over the devices instead")
    a = ap.parse_args()
    n = _lib.device_count()
    devs = [int(x) for x in a.devices.split(",")] if a.devices else list(range(n))
    dom = H.greenhouse_domain()
    N = dom.flat().n_emitters
    R = int(a.rays) // N
    kw = dict(seed=1, verbose=False, smooth=False, devices=devs if len(devs) > 1 else None, device=devs[0],
              bands=not a.rows)
    dom(R * N, **kw)  # uploads + warm-up
    best = None
    for _ in range(a.steps):
        t = time.perf_counter()
        dom(R * N, **kw)
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    info = sorted(dom.last_trace_info, key=lambda i: i["bin"])
    rays = sum(i["rays_traced"] for i in info)
    per = "  ".join(f"b{i['bin']} {i['trace_ms']:.1f}" for i in info)
    print(f"C5 {'rows' if a.rows else 'bands'} over devices {devs}: {len(info)} band traces, {rays:.3e} rays in {best * 1e3:.1f} ms "
          f"({rays / best / 1e9:.2f} Grays/s whole call)  kernel ms: {per}", flush=True)


if __name__ == "__main__":
    main()
