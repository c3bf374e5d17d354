"""Diagnostic: do back-to-back traces on two streams hide a launch's drain?

Loads librthx.so twice from two copies (RTLD_LOCAL: each instance keeps its
own per-device stream), uploads the BASELINE domain into each, and times K
enqueued (RTHX_FLAG_ASYNC) traces of 1e8 rays: all on one instance (one
stream, the bench's pipeline), then alternating the two instances (two
streams, two results).  Prints Grays/s of each and every result's checks.

  python tools/two_stream_probe.py --steps 40 --rounds 5
"""
import argparse
import ctypes as C
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytraceheattransfer.jl_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: F401,E402  (one HIP runtime for every instance)

from rthx import abi, _lib  # noqa: E402


def open_copy(src, tmp, tag):
    dst = os.path.join(tmp, f"librthx_{tag}.so")
    shutil.copy(src, dst)
    lib = C.CDLL(dst, mode=os.RTLD_LOCAL)
    lib.rthx_last_error.restype = C.c_char_p
    lib.rthx_domain_create.argtypes = [C.POINTER(abi.DomainDesc), C.c_int32, C.POINTER(C.c_void_p)]
    lib.rthx_result_create.argtypes = [C.POINTER(C.c_void_p)]
    lib.rthx_trace_exchange.argtypes = [C.c_void_p, C.POINTER(abi.TraceArgs), C.c_void_p]
    lib.rthx_result_get_info.argtypes = [C.c_void_p, C.POINTER(abi.ResultInfo)]
    lib.rthx_device_synchronize.argtypes = [C.c_int32]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--rays", type=int, default=100_000_000)
    ap.add_argument("--lib", default=os.path.join(ROOT, "raytraceheattransfer.jl_amd/csrc/_build/librthx.so"))
    args = ap.parse_args()
    import bench

    flat = bench.build_domain().flat()
    N = flat.n_emitters
    R = args.rays // N
    nudge = 10_000 * np.finfo(np.float64).eps
    targs, _k = _lib.make_args(0, R, nudge, 1, 0, N, 1, flags=abi.RTHX_FLAG_DEVICE_ONLY | abi.RTHX_FLAG_ASYNC)
    tmp = tempfile.mkdtemp(prefix="rthx2s_")
    inst = []
    for tag in ("a", "b"):
        lib = open_copy(args.lib, tmp, tag)
        h, r = C.c_void_p(), C.c_void_p()
        assert lib.rthx_domain_create(C.byref(flat.desc), 0, C.byref(h)) == 0, lib.rthx_last_error()
        assert lib.rthx_result_create(C.byref(r)) == 0
        inst.append((lib, h, r))

    def info(i):
        lib, _h, r = inst[i]
        inf = abi.ResultInfo()
        assert lib.rthx_result_get_info(r, C.byref(inf)) == 0, lib.rthx_last_error()
        return inf

    def run(order):
        for i in order:
            lib, h, r = inst[i]
            assert lib.rthx_trace_exchange(h, C.byref(targs), r) == 0, lib.rthx_last_error()
        inst[0][0].rthx_device_synchronize(0)

    for i in (0, 1):  # warm both instances (plans, occupancy, buffers)
        run([i] * 5)
        info(i)
    res = {"one stream": [], "two streams": []}
    for _ in range(args.rounds):
        for name, order in (("one stream", [0] * args.steps), ("two streams", [k & 1 for k in range(args.steps)])):
            t = time.perf_counter()
            run(order)
            el = time.perf_counter() - t
            checked = faults = 0
            for i in set(order):
                inf = info(i)
                checked += inf.superseded + 1
                faults += inf.superseded_faults + inf.lookback_fallbacks
                rays = inf.rays_traced
            assert checked == args.steps and faults == 0, (name, checked, faults)
            res[name].append(rays * args.steps / el / 1e9)
    for name, v in res.items():
        v = np.array(v)
        print(f"{name:12s} median {np.median(v):.2f} Grays/s  min {v.min():.2f}  max {v.max():.2f}  "
              f"({args.steps} steps of {rays} rays, {args.rounds} rounds; every step checked)", flush=True)
    shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    main()
