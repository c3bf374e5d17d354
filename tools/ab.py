"""A/B timing of several librthx.so builds in ONE process (diagnostic).

Each library is loaded with RTLD_LOCAL, gets its own domain and result on
device 0, and the libraries are timed in interleaved rounds so that clock and
thermal drift hit them alike.  Prints the median trace-kernel time (HIP
events) per library.

  python tools/ab.py --rays 100000000 --rounds 8 libA.so libB.so ...
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "raytraceheattransfer.jl_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: F401,E402  (one HIP runtime for all libraries)

from rthx import abi, _lib  # noqa: E402


def open_lib(path):
    lib = C.CDLL(path, mode=os.RTLD_LOCAL)
    lib.rthx_last_error.restype = C.c_char_p
    lib.rthx_domain_create.argtypes = [C.POINTER(abi.DomainDesc), C.c_int32, C.POINTER(C.c_void_p)]
    lib.rthx_result_create.argtypes = [C.POINTER(C.c_void_p)]
    lib.rthx_trace_exchange.argtypes = [C.c_void_p, C.POINTER(abi.TraceArgs), C.c_void_p]
    lib.rthx_result_get_info.argtypes = [C.c_void_p, C.POINTER(abi.ResultInfo)]
    return lib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--rays", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--ndim", type=int, default=101)
    ap.add_argument("--c5-bin", type=int, default=-1, help="time one band of the C5 greenhouse instead of C2")
    ap.add_argument("--stride", type=int, default=1,
                    help="rank 0's rows of a W-way row shard (rows 0, W, 2W, ...; --rays stays the whole job's)")
    ap.add_argument("--env", default="",
                    help="NAME=v1,v2,...: every library is also timed with each value of that knob "
                         "(RTHX_DEV_KNOBS is set; 'auto' leaves the knob unset)")
    ap.add_argument("--with-pack", action="store_true",
                    help="time trace + pack (staged rows: row scan, part merge, CSR pack) instead of the trace kernel alone")
    ap.add_argument("--sets", default="",
                    help="knob sets separated by '|', each 'NAME=v:NAME2=v2' ('none' = no knobs): every library is "
                         "also timed with each set (replaces --env)")
    args = ap.parse_args()
    import bench

    if args.c5_bin >= 0:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import helpers as H

        dom = H.greenhouse_domain()
    else:
        dom = bench.build_domain(args.ndim)
    flat = dom.flat()
    N = flat.n_emitters
    R = args.rays // N
    nudge = 10_000 * np.finfo(np.float64).eps
    targs, _k = _lib.make_args(max(args.c5_bin, 0), R, nudge, 1, 0, N, args.stride, flags=abi.RTHX_FLAG_DEVICE_ONLY)
    os.environ["RTHX_DEV_KNOBS"] = "1"
    knob, vals = (args.env.split("=", 1)[0], args.env.split("=", 1)[1].split(",")) if args.env else (None, [None])
    if args.sets:
        knob, vals = "sets", args.sets.split("|")
    set_names = set()
    for v in (vals if knob == "sets" else []):
        set_names |= {kv.split("=", 1)[0] for kv in v.split(":") if "=" in kv}

    def set_knob(v):
        if knob is None:
            return
        if knob == "sets":
            for k in set_names:
                os.environ.pop(k, None)
            for kv in v.split(":"):
                if "=" in kv:
                    k, x = kv.split("=", 1)
                    os.environ[k] = x
            return
        if v in (None, "auto"):
            os.environ.pop(knob, None)
        else:
            os.environ[knob] = v

    runs = []
    for p in args.libs:
        lib = open_lib(p)
        for v in vals:
            set_knob(v)
            h, r = C.c_void_p(), C.c_void_p()
            assert lib.rthx_domain_create(C.byref(flat.desc), 0, C.byref(h)) == 0, lib.rthx_last_error()
            assert lib.rthx_result_create(C.byref(r)) == 0
            for _ in range(2):
                assert lib.rthx_trace_exchange(h, C.byref(targs), r) == 0, lib.rthx_last_error()
            tag = os.path.basename(os.path.dirname(p)) or p
            label = f" [{v}]" if knob == "sets" else (f" {knob}={v}" if knob else "")
            runs.append((tag + label, lib, h, r, [], v))
    for _ in range(args.rounds):
        for p, lib, h, r, ts, v in runs:
            set_knob(v)
            for _ in range(args.steps):
                assert lib.rthx_trace_exchange(h, C.byref(targs), r) == 0
                inf = abi.ResultInfo()
                lib.rthx_result_get_info(r, C.byref(inf))
                ts.append(inf.trace_ms + (inf.pack_ms if args.with_pack else 0.0))
    rays = len(range(0, N, args.stride)) * R
    for p, lib, h, r, ts, v in runs:
        t = np.array(ts)
        print(f"{p:12s} median {np.median(t):.4f} ms  min {t.min():.4f}  "
              f"p90 {np.percentile(t, 90):.4f}  {rays / np.median(t) / 1e6:.1f} Mrays/s (R={R}, {rays // R} rows)", flush=True)


if __name__ == "__main__":
    main()
