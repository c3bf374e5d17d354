import sys, os, time
sys.path.insert(0, 'raytraceheattransfer.jl_amd'); sys.path.insert(0, '.')
import numpy as np, bench
from rthx import _lib, abi
dom = bench.build_domain(); flat = dom.flat(); N = flat.n_emitters; R = 100_000_000 // N
dd = _lib.DeviceDomain(flat, 0); res = _lib.DeviceResult()
a, _k = _lib.make_args(0, R, 10_000 * np.finfo(np.float64).eps, 1, 0, N, 1, flags=abi.RTHX_FLAG_DEVICE_ONLY)
ts = []
t0 = time.perf_counter()
for i in range(300):
    res.trace(dd, a); ts.append(res.info()['trace_ms'])
print('total s', time.perf_counter() - t0)
ts = np.array(ts)
for i in range(0, 300, 10): print(i, np.round(ts[i:i+10], 3).tolist())
