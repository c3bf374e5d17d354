"""Diagnostic: rows where the device and the CPU restatement disagree on a
layered slab (tests/helpers.layered_slab_domain)."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "raytraceheattransfer.jl_amd"), ROOT]
import numpy as np
import helpers as H
from oracle import oracle
from rthx import _lib

for ks in ([4.0, 0.0, 0.0, 0.0], [0.0, 0.0, 0.0, 4.0], [4.0, 1e-3, 1e-3, 1e-3], [2.0, 0.0, 2.0]):
    dom = H.layered_slab_domain(ks)
    flat = dom.flat()
    N = flat.n_emitters
    args, _k = _lib.make_args(0, 20000, H.NUDGE, 11, 0, N, 1)
    dd = _lib.DeviceDomain(flat, 0)
    res = _lib.DeviceResult()
    res.trace(dd, args)
    info = res.info()
    rp, c, n = res.csr()
    res.close(); dd.close()
    orp, oc, on, oi, _ = oracle.trace_exchange(flat, args, 16)
    bad = [g for g in range(N) if not (np.array_equal(c[rp[g]:rp[g+1]], oc[orp[g]:orp[g+1]]) and np.array_equal(n[rp[g]:rp[g+1]], on[orp[g]:orp[g+1]]))]
    print(ks, "N", N, "surfaces", dom.num_surfaces, "lost gpu/oracle", info["lost_total"], oi["lost_total"], "bad rows", len(bad), bad[:12])
    for g in bad[:3]:
        a = dict(zip(c[rp[g]:rp[g+1]].tolist(), n[rp[g]:rp[g+1]].tolist()))
        b = dict(zip(oc[orp[g]:orp[g+1]].tolist(), on[orp[g]:orp[g+1]].tolist()))
        d = {k: (a.get(k, 0), b.get(k, 0)) for k in sorted(set(a) | set(b)) if a.get(k, 0) != b.get(k, 0)}
        print("   row", g, "diffs (col: gpu, oracle)", list(d.items())[:10])
