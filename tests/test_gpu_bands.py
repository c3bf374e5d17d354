"""BASELINE config C5 over W GPUs, row-sharded and pipelined, on the MI355X
(rthx.distributed.trace_bands_row_sharded, rthx_merge_row_shards).

Every rank traces its rows g = k, k + W, ... of every band; band i is
gathered to rank i mod W and merged there in row order by the HIP merge
kernels.  The counts of every merged band must equal the one-device trace of
the whole band bit for bit (the reference traces the bins one after another
on one host, parallelRayTracing.jl:20-42; the counter-based RNG makes a
row's counts independent of who traces it).  One GPU holds one NCCL rank, so
W > 1 runs as the one-GPU emulation (each emulated rank's peers' blocks
traced beforehand on the same GPU, EmulatedBandComm); the NCCL (RCCL) branch
runs on a one-rank group.
"""
import socket

import numpy as np
import pytest

import helpers as H

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _full_band(hip, dd, flat, b, R, seed):
    args, _k = hip.make_args(b - 1, R, H.NUDGE, seed, 0, flat.n_emitters, 1)
    res = hip.DeviceResult()
    try:
        res.trace(dd, args)
        return res.csr()
    finally:
        res.close()


@pytest.mark.parametrize("W", [1, 2, 3, 8, 64])
def test_merge_row_shards_device_exact(hip, W):
    """W strided row blocks traced on the GPU, merged on the GPU, equal the
    whole trace (W = 64: the ABI's largest shard count, blocks of 2-3 rows)."""
    from rthx.distributed import HipShardTracer, merge_row_shards_device

    dom = H.square_domain(11, kappa=0.7)
    flat = dom.flat()
    N, R = flat.n_emitters, 3001
    tracer = HipShardTracer(dom, 0, n_results=1)
    ros, cs, ns = [], [], []
    try:
        for k in range(W):
            sh = tracer(0, R, H.NUDGE, 5, k, W, False)
            ro = torch.empty(sh.n_rows + 1, dtype=torch.int64, device="cuda:0")
            pr = torch.empty((2, max(sh.nnz, 1)), dtype=torch.int32, device="cuda:0")
            sh.fill(ro, pr[0], pr[1])
            sh.done()
            ros.append(ro)
            cs.append(pr[0])
            ns.append(pr[1])
    finally:
        tracer.close()
    rp, c, v = merge_row_shards_device(ros, cs, ns, N)
    torch.cuda.synchronize()
    frp, fc, fv = _full_band(hip, hip.DeviceDomain(flat, 0), flat, 1, R, 5)
    assert np.array_equal(rp.cpu().numpy(), frp)
    assert np.array_equal(c.cpu().numpy(), fc)
    assert np.array_equal(v.cpu().numpy().view(np.uint32), fv)


def _check_owned(hip, dom, owned, info, R, seed, rank):
    flat = dom.flat()
    dd = hip.DeviceDomain(flat, 0)
    try:
        mine = {b for b, o in info["owner"].items() if o == rank}
        assert set(owned) == mine
        for b, (rp, c, v) in owned.items():
            frp, fc, fv = _full_band(hip, dd, flat, b, R, seed)
            assert np.array_equal(rp.cpu().numpy(), frp), b
            assert np.array_equal(c.cpu().numpy(), fc), b
            assert np.array_equal(v.cpu().numpy().view(np.uint32), fv), b
    finally:
        dd.close()


@pytest.mark.parametrize("W,overlap,last_parts", [(3, True, 2), (2, False, 1), (2, True, 3)])
def test_row_sharded_pipeline_emulated_ranks_exact(hip, W, overlap, last_parts):
    """Every emulated rank of W runs the whole pipeline (its rows of all 8
    bands traced, its bands' blocks gathered and merged on the GPU): each
    merged band equals the one-device trace."""
    from rthx.distributed import EmulatedBandComm, trace_bands_row_sharded

    dom = H.greenhouse_domain(n_layers=4, nx=9, ny=3, n_bins=8)
    N = dom.flat().n_emitters
    R, seed = 1200, 7
    seen = set()
    for q in range(W):
        comm = EmulatedBandComm.for_rank(dom, R * N, q, W, 0, seed=seed, nudge=H.NUDGE, last_parts=last_parts)
        owned, info = trace_bands_row_sharded(dom, R * N, seed=seed, nudge=H.NUDGE, overlap=overlap, comm=comm,
                                              last_parts=last_parts)
        assert len(info["traces"]) == 7 + last_parts
        assert sum(t["rows_traced"] for t in info["traces"][7:]) == len(range(q, N, W))
        assert all(t["rows_traced"] == len(range(q, N, W)) for t in info["traces"][:7])
        _check_owned(hip, dom, owned, info, R, seed, q)
        seen |= set(owned)
    assert len(seen) == 8


def test_row_sharded_pipeline_over_rccl(hip):
    """The product branch: TorchBandComm on an NCCL (= RCCL) group, one rank
    (a one-GPU box holds one), all 8 bands assembled on it."""
    import torch.distributed as dist

    from rthx.distributed import trace_bands_row_sharded

    dom = H.greenhouse_domain(n_layers=4, nx=9, ny=3, n_bins=8)
    N = dom.flat().n_emitters
    R, seed = 1500, 3
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        owned, info = trace_bands_row_sharded(dom, R * N, seed=seed, nudge=H.NUDGE)
        assert all(o == 0 for o in info["owner"].values())
        assert all(rp.device.type == "cuda" for rp, _c, _v in owned.values())
        _check_owned(hip, dom, owned, info, R, seed, 0)
    finally:
        dist.destroy_process_group()
