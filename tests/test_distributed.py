"""World-size-2 gloo rehearsal of the multi-GPU path on the CPU: every rank
traces its strided emitter rows (here with the CPU oracle standing in for the
device, test infrastructure only), rank 0 gathers the disjoint CSR row blocks
(rthx.distributed.gather_csr) and must reproduce the single-process F exactly
(the counter-based RNG makes rows independent of the rank that traced them)."""
import os
import socket
import sys

import numpy as np
import pytest

import helpers as H

torch = pytest.importorskip("torch")
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    sys.path[:0] = [H.PKG, H.ROOT, os.path.join(H.ROOT, "tests")]
    import torch.distributed as dist

    from oracle import oracle
    from rthx import _lib
    from rthx.distributed import gather_csr, shard

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dom = H.wedge_domain(8, 3)
    flat = dom.flat()
    begin, stride = shard(rank, world)
    args, _k = _lib.make_args(0, 500, H.NUDGE, 9, begin, flat.n_emitters, stride)
    rp, cols, cnt, info, _ = oracle.trace_exchange(flat, args, 2)
    merged = gather_csr(rp, cols, cnt, flat.n_emitters)
    if rank == 0:
        np.savez(out_path, row_ptr=merged[0], cols=merged[1], counts=merged[2])
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gather_equals_single_process(tmp_path):
    out = str(tmp_path / "merged.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    from oracle import oracle
    from rthx import _lib

    dom = H.wedge_domain(8, 3)
    flat = dom.flat()
    args, _k = _lib.make_args(0, 500, H.NUDGE, 9, 0, flat.n_emitters, 1)
    rp, cols, cnt, _info, _ = oracle.trace_exchange(flat, args, 4)
    m = np.load(out)
    assert np.array_equal(m["row_ptr"], rp)
    assert np.array_equal(m["cols"], cols)
    assert np.array_equal(m["counts"], cnt)


def _direct_worker(rank, world, port, out_path):
    """method=:direct sharded by ray range; the per-element counts are summed
    with an all-reduce (rthx.direct, distributed=True)."""
    sys.path[:0] = [H.PKG, H.ROOT, os.path.join(H.ROOT, "tests")]
    import torch.distributed as dist

    from oracle import oracle
    from rthx import direct as DR

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dom = H.square_domain(5, kappa=0.5, sigma_s=0.5, epsilon=0.7)
    counts, total, info = DR.direct_ray_tracing_single_bin(dom, 30_001, H.NUDGE, 1, seed=5,
                                                           backend=oracle.OracleBackend(2), distributed=True)
    assert info["rays_traced"] == DR.ray_shard(rank, world, 30_001)[1] - DR.ray_shard(rank, world, 30_001)[0]
    if rank == 0:
        np.save(out_path, counts)
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_direct_allreduce_equals_single_process(tmp_path):
    out = str(tmp_path / "direct.npy")
    mp.spawn(_direct_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    from oracle import oracle
    from rthx import direct as DR

    dom = H.square_domain(5, kappa=0.5, sigma_s=0.5, epsilon=0.7)
    counts, _total, _info = DR.direct_ray_tracing_single_bin(dom, 30_001, H.NUDGE, 1, seed=5,
                                                             backend=oracle.OracleBackend(4))
    assert np.array_equal(np.load(out), counts)
